// Front end of the configs[4] training step (train_front.hip): embedding, encoder convolutions
// and bidirectional Zoneout-LSTM, both reference encoders (conv2d + BN + ReLU, GRU, dense) and
// both GST attentions, forward in training mode and backward.  Elementwise / recurrent kernels
// here; every matrix product goes through gemm.hip from train.hip's orchestration.
#pragma once
#include "common.h"

namespace tt2 {

// ---- encoder --------------------------------------------------------------------------------
void fe_embed(const int* ids, const float* table, long M, int E, float* out, hipStream_t s);
// scratch (>= min(64, M/128) x n_symbols x E floats, or null): the position-segmented two-pass form
void fe_embed_bwd(const int* ids, const float* dx, long M, int E, int n_symbols, float* dtable, hipStream_t s,
                  float* scratch = nullptr, long scratch_floats = 0);

// BiLSTM step t of both directions (bidirectional_dynamic_rnn, modules.py:315-321): layouts are
// direction-major: XP [B][T][8U] input projections (+ biases), GZ [2][B][4U] recurrent products of
// this step, GA [2][T][B][4U] activations (σi, tanh j, σ(f+1), σo), CN [2][T][B][U] c_new,
// CS / HS [2][T+1][B][U] carried (zoned) states, ENC [B][T][2U] outputs (h_new, 0 past length).
// zm [T][2][2][B][U] training zoneout keep bits (c, h) by step, or null (inference mix).
struct FeLstm {
  const float* XP; const float* GZ; float* GA; float* CN; float* CS; float* HS; float* ENC;
  const uint8_t* zm; const int* lens;
  int B, T, U, t;
  float zo;
  // backward
  const float* DENC; long ld_denc;  // d enc_out rows (stride ld_denc, the decoder's d memory)
  float* DZ;                        // [2][T][B][4U]
  float* DHC; float* DCC;           // [2][B][U] gradient wrt the carried h / c after step t
  float* DHP;                       // [2][B][U] direct part of d h_prev (before + DZ·Whᵀ)
};
void fe_lstm_cell(const FeLstm& a, hipStream_t s);
void fe_lstm_cell_bwd(const FeLstm& a, hipStream_t s);
// dXP[b][pos][dir*4U + c] = DZ[dir][t][b][c] at the step that visited pos (0 past length)
void fe_lstm_dxp(const float* DZ, const int* lens, int B, int T, int U, float* dXP, hipStream_t s);

// ---- reference encoder ----------------------------------------------------------------------
// BN (batch statistics) + ReLU forward; backward sums use the post-ReLU output as the ReLU mask
void fe_bn_relu_fwd(const float* a, long M, int C, const float* mean, const float* var, const float* gamma,
                    const float* beta, float eps, float* y, hipStream_t s);
void fe_relu_mask(const float* dy, const float* y, long n, float* out, hipStream_t s);
// conv2d 3x3 stride st (2, or 1 for ReferenceEncoderAdaIn's deeper layers) 'same' (TF: odd pad
// bottom/right) on NHWC x [N][H][W][C]
void fe_im2col2d_t(const float* x, int N, int H, int W, int C, int Ho, int Wo, int pt, int pl, float* out, long ldo,
                   hipStream_t s, int st = 2);
void fe_col2im2d(const float* dcols, int N, int H, int W, int C, int Ho, int Wo, int pt, int pl, float* dx,
                 hipStream_t s, int st = 2);
// the same conv2d's backward without a materialised im2col (fp32 FMA): the kernel gradient as
// partial rows [rows][9·C·F] into part (returns rows; the caller sums them), the input gradient as a
// gather over the taps.  *_ok: the channel counts these kernels take (LDS / register budgets)
// forward of the same conv2d for C <= 4 input channels (the refnets' first layer): + bias, optional ReLU;
// bf16: operands rounded to bf16 as the bf16 step's GEMM form rounds them
bool fe_conv2d_fwd_small_ok(int C, int F);
void fe_conv2d_fwd_small(const float* x, const float* Wk, const float* bias, int N, int H, int W, int C, int Ho, int Wo,
                         int F, int pt, int pl, int st, bool relu, float* out, hipStream_t s, bool bf16);
bool fe_conv2d_dw_ok(int C, int F);
int fe_conv2d_dw(const float* x, const float* dz, int N, int H, int W, int C, int Ho, int Wo, int F, int pt, int pl,
                 int st, float* part, long part_floats, hipStream_t s);
bool fe_conv2d_dx_ok(int C, int W, int Ho, int Wo, int F, int st);
void fe_conv2d_dx(const float* dz, const float* Wk, int N, int H, int W, int C, int Ho, int Wo, int F, int pt, int pl,
                  int st, float* dx, hipStream_t s);
// ReferenceEncoderAdaIn (modules.py:89-98): per (row, channel) moments of NHWC x over HW -> mv [N][C][2]
// (mean, biased variance); the 0.9 / 0.1 restyle of the speaker map by the emotion map's moments and
// its backward (S: [N][C][2] scratch; dxe: the emotion map's gradient through m_e, v_e)
void fe_ad_moments(const float* x, int N, int HW, int C, float* mv, hipStream_t s);
void fe_ad_mix(const float* xs, int N, int HW, int C, const float* mv_s, const float* mv_e, float* y, hipStream_t s);
void fe_ad_mix_bwd(const float* dy, const float* xs, const float* xe, int N, int HW, int C, const float* mv_s,
                   const float* mv_e, float* S, float* dxs, float* dxe, hipStream_t s);
// GRU (TF1 GRUCell, modules.py:59): XG [N][T2][3D] = x·[Wg_x | Wc_x] + [bg | bc]; per step
// GG = h·Wg_h [N][2D], GC = (r·h)·Wc_h [N][D]; stored step-major R, U, CC [T2][N][D], RH [T2][N][D],
// HG [T2+1][N][D]
void fe_gru_a(const float* XG, const float* GG, const float* HG, int N, int T2, int D, int t, float* R, float* Uu,
              float* RH, hipStream_t s);
void fe_gru_b(const float* XG, const float* GC, const float* Uu, int N, int T2, int D, int t, float* CC, float* HG,
              hipStream_t s);
// backward of step t: dH [N][D] in (gradient wrt h(t+1)); writes DCP[t] (pre-tanh candidate grad),
// DHA = dh·u; then (after the d(r·h) product) DGP[t] and DHA += d(rh)·r
// the whole recurrence of one reference encoder's GRU in one work-group (N <= 64, RD 32 / 128): the same
// outputs as the per-step fe_gru_a / fe_gru_b (forward) and fe_gru_bwd_a / b + the two products
// (backward; dH holds d h(T2) on entry and d h(0) on exit).  Wgh = the gates kernel's h rows [RD][2RD],
// Wch = the candidate kernel's h rows [RD][RD]; bf16: bf16 operands (the bf16 step), else fp32 MFMA
bool fe_gru_seq_ok(int N, int RD);
void fe_gru_fwd_seq(const float* XG, const float* Wgh, const float* Wch, int N, int T2, int RD, float* R, float* Uu,
                    float* RH, float* CC, float* HG, hipStream_t s, bool bf16 = false);
void fe_gru_bwd_seq(const float* Wgh, const float* Wch, const float* R, const float* Uu, const float* CC, const float* HG,
                    int N, int T2, int RD, float* dH, float* DCP, float* DGP, hipStream_t s, bool bf16 = false);
void fe_gru_bwd_a(const float* dH, const float* Uu, const float* CC, const float* HG, int N, int D, int t, float* DCP,
                  float* DHA, hipStream_t s);
void fe_gru_bwd_b(const float* DRH, const float* R, const float* Uu, const float* HG, const float* CC, const float* dH,
                  int N, int D, int t, float* DGP, float* DHA, hipStream_t s);
// DXG [N][T2][3D] (row n*T2 + t) from step-major DGP [T2][N][2D] / DCP [T2][N][D]
void fe_gru_dxg(const float* DGP, const float* DCP, int N, int T2, int D, float* DXG, hipStream_t s);
void fe_tanh_bwd(const float* dy, const float* y, long n, float* out, hipStream_t s);

// ---- GST multi-head attention (multihead_attention.py:35-132, mlp attention, normalize) -------
struct FeGst {
  const float* ref;     // [N][128] reference embedding
  const float* tokens;  // [ntok][tokd]
  const float* wq; const float* bq;  // [128][A], [A]
  const float* wk; const float* bk;  // [tokd][A], [A]
  const float* v; const float* g; const float* bb;  // [A/heads], scalar, [A/heads]
  int N, ntok, tokd, A, heads, refd;
  float* style; int style_ld, style_off;  // output [N][style_ld] at column style_off (heads*tokd wide)
  // backward
  const float* dstyle;   // [N][style_ld] (same column window)
  float* dq;             // [N][A]
  float* pdkk;           // [N][ntok][A]
  float* pdv;            // [N][ntok][tokd]  (value path)
  float* pdnv;           // [N][A/heads]
  float* pdbb;           // [N][A/heads]
};
void fe_gst_fwd(const FeGst& a, hipStream_t s);
void fe_gst_bwd(const FeGst& a, hipStream_t s);
// from the row-summed partials: d Wk, d bk, d tokens, d v, d g, d attention_b
void fe_gst_final(const FeGst& a, const float* dkk, const float* dval, const float* dnv, const float* dbb,
                  float* dwk, float* dbk, float* dtok, float* dv, float* dg, float* dbbo, hipStream_t s);

// ---- memory assembly --------------------------------------------------------------------------
// MEM[b][t] = [ENC[b][t] (2U) | STY[b] (SW)]; style gradient = Σ_t DMEM[b][t][2U:]
void fe_memory(const float* ENC, const float* STY, int B, int T, int E2, int SW, float* MEM, hipStream_t s);
void fe_style_grad(const float* DMEM, int B, int T, int D, int E2, float* DSTY, hipStream_t s);

}  // namespace tt2
