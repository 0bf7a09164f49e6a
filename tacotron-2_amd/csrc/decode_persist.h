// Persistent Tacotron-2 decoder (gfx950): the whole dynamic_decode loop as ONE launch of 256
// work-groups (one per CU) with the recurrent weights resident in registers and LDS.  See
// decode_persist.hip for the schedule and DESIGN.md §5 for the roofline.
#pragma once
#include "common.h"

namespace tt2 {

// Fixed geometry of the persistent path (fork-default hparams, hparams.py:147-178).  Other shapes
// run the per-step launch path in tacotron.hip.
constexpr int PD_NB = 256;    // work-groups = LSTM column tiles (4 hidden units x 4 gates each)
constexpr int PD_NT = 512;    // threads per work-group (8 waves, 2 per SIMD)
constexpr int PD_H = 1024;    // decoder_lstm_units
constexpr int PD_P = 256;     // prenet_units
constexpr int PD_E2 = 512;    // encoder-output half of the attention memory
constexpr int PD_A = 128;     // attention_dim
constexpr int PD_NPJ = 96;    // frame (80) + stop (1) columns, padded to 16
constexpr int PD_NPF = 352;   // + the prenet-L1 columns folded into the projection
constexpr int PD_NTILE = 22;  // projection column tiles
constexpr int PD_KSP = 8;     // projection K split (128 h2 rows + 64 context rows per split)
constexpr int PD_TMAX = 256;  // encoder steps of the values slice held in registers (k_decode_persist<., 256>)
constexpr int PD_TMAX_LONG = 512;  // max encoder steps: T_in > 256 runs k_decode_persist<false, 512>
constexpr int PD_KLP = 32;    // location-conv taps padded to 16
constexpr int PD_NREP = 8;    // replicas of the H1/H2 flag lines (32 pollers per line)
// Hidden unit q (0..3) of LSTM tile g: the four units of a tile are the four components of one AF
// float4 (common.h af_idx), 16(g/4) + g%4 + 4q.  Tiles [32w, 32w+32) own units [128w, 128w+128).
__host__ __device__ inline int pd_unit(int g, int q) { return 16 * (g >> 2) + (g & 3) + 4 * q; }
enum { PD_F_PRE = 0, PD_F_H1, PD_F_H2, PD_F_E, PD_F_CTX, PD_F_PP, PD_F_QE, PD_F_CMB, PD_F_EO, PD_F_EMT, PD_NPH };
// Tacotron_emt_attn 'multihead' / 'style_tokens' in the persistent decoder (k_decode_persist<true>): the
// emotion query (128) rides as 8 more projection tiles; 16 emotion work-groups own 2 rows each; the
// attn_emt dense (KC -> 128, 'multihead' only) runs on the 64 emotion-query projection work-groups.
constexpr int PD_ENT = 8;        // emotion-query projection tiles (128 = style_att_dim)
constexpr int PD_EG0 = 240;      // first emotion work-group (rows 2(g-240), +1)
constexpr int PD_EQ = 128;       // emotion query width = attn_emt dense output width

struct PdArgs {
  unsigned* flags;  // [PD_NPH][PD_NB] hand-off tags (zeroed before every launch)
  unsigned* flags2; // [PD_NPH][8 groups][32] group-level tags of the all-producer waits
  int* ctl;         // [4]: done, n_steps, err, pad (zeroed before every launch)
  unsigned* rflags; // [3: H1, H2, EMT][PD_NREP replicas][PD_NB] hand-off tags, one replica per consumer XCD group
  int B, T_in, max_iters, T_lim, nm;
  int stop_at_any, mask_encoder, cumulative, constraint, monotonic, win;
  float zo, one_m_zo;
  int poll_sleep;       // s_sleep(1) repetitions between flag polls (env TT2_PD_SLEEP)
  // weights (tacotron.hip finalize layouts)
  const float* l1_w;    // [256 tiles][768 x 16] WF, rows [prenet | context_enc]
  const float* l1_wh;   // [256][1024 x 16] recurrent rows
  const float* l1_b;    // [4096] lstm column order
  const float* l2_w;    // [256][1024 x 16] input rows (h1_new)
  const float* l2_wh;   // [256][1024 x 16] recurrent rows
  const float* l2_b;
  const float* GS;      // [32][4096] style·W1[style rows] per utterance
  const float* q_wt;    // [128][1024] query_layer kernel, transposed
  const float* loc_cw;  // [8 tiles][32 x 16] WF (location conv folded through the location dense)
  const float* va;      // [128] attention_variable_projection
  const float* proj_w;  // [22 tiles][1536 x 16] WF, rows [h2 | context_enc]
  const float* proj_b;  // [352]
  const float* PS;      // [32][352] style·W_proj[style rows]
  const float* pre_b1;  // [256] prenet L1 bias, AF-group column order
  const float* pre_w2t; // [256 out][256 in] prenet layer-2 kernel, transposed
  const float* pre_b2;  // [256]
  const float* TP1;     // GTA: [B][T_lim][256] targets·W1 + b1 (AF-group order), or null
  const float* keysT;   // [B][128][TM] keys (+ b_a + b_conv·W_loc), encoder step fastest (TM = 256 | 512)
  const float* valuesT; // [B][512][TM] encoder half of the values, encoder step fastest, 0 past T_in
  const int* lengths;   // [B]
  const uint8_t* masks; // [max_iters][2][B][256] prenet keep bits
  // exchange buffers, two step parities each
  float* H1x;   // [2][32 x 1024] AF: h1_new
  float* H2x;   // [2][32 x 1024] AF: h2_new
  unsigned long long* Eg;  // [2][32 rows][8 slices][TM t] {tag, partial energy} granules
  float* CTXx;  // [2][32 x 512] AF: context_enc
  float* SSx;   // [2][32]: Σ_{t<len} alignments (style-context scale)
  unsigned long long* PPg; // [2][8 splits][32 rows][352] {tag, projection partial} granules
  unsigned long long* PREg;  // [2][32 x 256] AF-ordered {tag = step<<1 | stop bit, prenet output} granules
  // outputs
  float* frames;  // [B][max_iters][nm]
  float* stop;    // [B][max_iters]
  float* align;   // [B][max_iters][T_in] step-major (tacotron.hip transposes after the launch) or null
  long long* stamps;  // diagnostic s_memrealtime stamps of one step (null = off)
  int stamp_step;
  // Tacotron_emt_attn 'multihead' (k_decode_persist<true> only)
  int K1;               // LSTM-1 critical rows per tile: P + E2 (+ 128 emotion block)
  int e_Tv, e_Dv, e_KC, e_heads, e_dh;  // attended rows, value width, heads x Dv, heads, dims per head
  int e_dense;          // 1 'multihead': contexts -> attn_emt dense (+ refnet_spk) = the block; 0 'style_tokens':
                        // the heads-concatenated contexts are the block
  int e_XW;             // block width joining LSTM-1 (128 'multihead', 64 'style_tokens')
  long e_vbs, e_kbs;    // batch strides of e_val / e_ke (0: style tokens shared by every row)
  int e_simple;         // 'simple' (SimpleBahdanauAttention): one softmax per row over V(tanh(W1 v + W2 q))
                        // computed as e_heads unit-slice partials; the context (Dv = 128) is the block
  const float* e_spk1;  // [32][4096] refnet_spk·W1[speaker rows] in lstm-column order ('simple': the
                        // speaker half of the concatenated block, constant per row -> LSTM-1 bias), or null
  const float* e_ke;    // [B][Tv][128] keys of the attended values (conv1d_1 + bias)
  const float* e_val;   // [B][Tv][Dv] attended values
  const float* e_qrow;  // [32][128] query bias per row
  const float* e_vv;    // [dh] g·v/|v|
  const float* e_ab;    // [dh] attention_b
  const float* e_wd;    // [8 tiles][KC x 16] WF (x KG_SB): attn_emt dense kernel
  const float* e_bd;    // [128] its bias
  const float* e_spk;   // [B][128] refnet_spk (added to the dense output), or null
  float* e_hist;        // [max_iters][B][heads][Tv] emotion alignments
  unsigned long long* QEg;  // [2][8 K splits][32][128] emotion-query partial granules (x KG_SB)
  float* CMBx;          // [2][32 x KC] AF emotion contexts (heads concatenated)
  unsigned long long* EOg;  // [2][8 K splits][32][128] dense partial granules (x KG_SB)
  float* EMTx;          // [2][32 x 128] AF emotion block of the next step's LSTM-1 input
};

size_t pd_lds_bytes();
// True when this device can keep all PD_NB work-groups resident at once.
bool pd_device_ok(int dev);
// tm: 256, or 512 for T_in > 256 (no emotion attention)
void pd_launch(const PdArgs& a, hipStream_t s, bool emt = false, int tm = PD_TMAX);

}  // namespace tt2
