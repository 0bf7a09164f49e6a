// Teacher-forced Tacotron-2 decoder training step (BASELINE configs[4]).
//
// One call = TacoTrainingHelper(ratio 1) dynamic_decode forward (helpers.py:62-133,
// Architecture_wrappers.py:197-267) with every activation kept resident in HBM, the losses of the
// slice (before-MSE tacotron.py:774, stop sigmoid CE :778-779, L2 :865-867), backpropagation
// through time, and (separately) clip_by_global_norm(1.0) + Adam (tacotron.py:1029,1219-1221).
//
// Layout (time-major, t = decoder step, b = row; one slot per step, slot T is the carry-out):
//   X1[t]  [B, P + D + H]   LSTM-1 input  [prenet(target_{t-1}) | ctx_{t-1} | hz1_{t-1}]
//   X2[t]  [B, 2H]          LSTM-2 input  [h1_new_t | hz2_{t-1}]
//   PIN[t] [B, H + D]       projection input [h2_new_t | ctx_t]
//   G*[t]  [B, 4H]          gate activations (σi, tanh j, σ(f+1), σo) after the forward
//   ALIGN  [B, T_in, T]     alignments (row-major per utterance: the d_values GEMM reads it as A)
// Every matrix product is an MFMA GEMM from gemm.hip (fp32 operands, or bf16 operands with fp32
// accumulation when cfg.precision = 1): per-step products at M = B with split-K (the LSTM cells
// fused into the split-K combine, gemm_raw), the weight gradients as one GEMM over all T·B rows
// after the loop (activations transposed once).  The recurrences' elementwise parts (LSTM cells,
// location-sensitive attention, softmax, context) and the Postnet's training-mode batch norm are
// the kernels below.  Backward mirrors the forward slot layout: dX1[t], dX2[t] hold the gradients
// of the step-t inputs, so a step's carry-ins are read from slot t+1.
#include <cmath>
#include <cstring>
#include <functional>


#include "common.h"
#include "gemm.h"
#include "train_front.h"
#include "train_bwd_persist.h"
#include "train_persist.h"

namespace tt2 {

struct TrVar {
  std::string name;
  std::vector<int64_t> shape;
  long off = 0, n = 0;
  bool reg = false;
};

}  // namespace tt2

using namespace tt2;

struct tt2_train_ctx {
  int dev = 0;
  hipStream_t stream = nullptr;
  tt2_train_config cfg{};
  int B = 0, Tm = 0, Tin = 0, D = 0, NM = 0, P = 0, H = 0, A = 0, F = 0, KW = 0;
  int LX1 = 0;  // P + D + H
  int R = 1;    // outputs_per_step: frames per decoder step
  std::vector<TrVar> vars;
  std::map<std::string, int> index;
  long total = 0;
  WeightMap host;
  bool finalized = false;
  long step_count = 0;
  // flat parameter / gradient / Adam buffers
  DevBuf params, grads_own, adam_m, adam_v;
  float* grads = nullptr;  // grads_own or a caller-bound buffer
  // transposed weights (refreshed every step)
  DevBuf K1T, K2T, WqT, WfT, WsT, WmT, Wp2T;
  // activations
  DevBuf values, keys, X1, X2, PIN, G1, G2, C1, C2, CN1, CN2, Q, ALIGN, CUM, P1, XIN, FR, ST;
  // backward
  DevBuf dFR, dST, dPIN, dX1, dX2, dG1, dG2, DC1, DC2, R1, R2, DQ, DCTX, DKEYS, DCUM;
  DevBuf dV, dBA, dKC, dBC, DVAL, DMEM, dZ, dPre, TBUF, part, red, kpart;
  DevBuf DF2, DCUM2, PQ2, SC2;
  DevBuf DWGP;  // [B][NT][32][A] k_tr_att_bwd_q's d W_loc accumulators (TrAtt::DWGP)
  DevBuf SS;   // [T][B] smoothing: Σ sigmoid(e) per step (TrAtt::SS)
  DevBuf DWG;  // [32][A] k_tr_dwloc_cum: Σ cum_{t-1}·du per tap (+ the Σ du row)  // k_tr_att_bwd_q: df / d cum / d query / Σ a·d cum partials by step parity
  DevBuf TH, E, DF, PQ, FALL, ALN;
  // the large plain products (tr_gemm_big)
  DevBuf blasA, blasB, blasP;  // gemm_bf16_kc: bf16 operand copies, split-K partials
  bool fe_direct = true;  // TT2_FE_CONV_DIRECT=0 at create: the refnet conv2d backward as im2col + GEMM + col2im
  bool fe_gru_seq = true;  // TT2_FE_GRU_SEQ=0 at create: the refnet GRU as per-step launches (4 per step)
  bool blas_on = true;  // TT2_TRAIN_BLAS=0 at create: the large products on gemm_x3_kernel too
  long blas_calls = 0;
  // bf16 copies of the recurrent weights in both layouts (precision = bf16), refreshed per step
  DevBuf hK1, hK1T, hK2, hK2T, hWq, hWqT;
  DevBuf X1h, X2h;  // bf16 shadows of the X1 / X2 rows (inputs of the fused LSTM products)
  DevBuf dGh;       // bf16 shadows of one step's dG2 | dG1 rows (fused backward products)
  DevBuf tK1T, tK2T, tWq, tK2, tK1;  // the fused products' weights in TF layout (k_tr_tf_weights)
  // Postnet training (cfg.postnet): PA[i] activations (pre-BN), PX[i] layer inputs (PX[0] unused:
  // layer 1 reads the clipped frames), batch stats, projection, scratch
  DevBuf PA[8], PX[9];  // postnet_layers <= 8
  DevBuf BNM, BNV, PPRJ, dPP, DYb, DZb, dPXa, dPXb, WFLIP, PWT, CLIPM, pn_part;
  int PL = 0, PC = 0, PK = 0;
  bool pn_masks = false;
  int T_last = 0, Tin_last = 0;  // decoder steps / encoder positions of the last forward_backward
  int Tf_last = 0;               // its frame count T_last * R
  DevBuf FRT;                    // R > 1: the clipped frames time-major [T_f][B][NM] (the Postnet's input)
  bool pn_ran = false;  // batch stats of the last forward are valid (moving averages in apply)
  // bf16 Postnet convolutions over padded planes (gemm.h conv_bf16_planes): the layer input / dz
  // planes (pad rows zeroed when the shape changes) and the transposed bf16 weights of one layer
  DevBuf pnPl, pnWt;
  DevBuf fePl, feWt;  // the same for the text encoder's convolutions (TT2_PN_PLANES gates both)
  int fe_pl_B = -1, fe_pl_T = -1;
  DevBuf values16;         // bf16 values for the per-step context / d align reads (TT2_TR_VALUES16)
  bool values16_on = true;
  int pn_pl_B = -1, pn_pl_T = -1;
  bool pn_planes = false;
  hipStream_t last_stream = nullptr;  // stream of the last forward_backward / apply (read-backs)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = 0.f;
  // front end (cfg.frontend: encoder + reference encoders + GST, train_front.hip)
  int f_nref = 0, f_gin = 0, f_T2 = 0, f_T2max = 0;
  bool f_ran = false;
  // cfg.adain (ReferenceEncoderAdaIn, modules.py:66-107): stacks r = 0 (emotion mel) and r = 1 (speaker
  // mel) without batch norm, the speaker map restyled by the emotion map's moments, one GRU + dense
  // (r = 1 buffers): fADX the restyled map (GRU input), fADM moments [2 (emt, spk)][B][C][2], fADS the
  // backward's per-channel sums, fDYE the emotion stack's map gradient
  bool f_adain = false;
  DevBuf fADX, fADM, fADS, fDYE;
  DevBuf fTWf, fTWb, fHSh, fDZh;  // encoder BiLSTM fused steps: TF-layout weights and state / dZ shadows
  DevBuf fEX, fEA[8], fEY[9], fXP, fGZ, fGA, fCN, fCS, fHS, fENC, fMEM, fSTY, fDSTY, fDZ, fDHC, fDCC, fDHP, fdXP, fdA,
      fdB, fLWxT, fLWhT;
  DevBuf fRA[2][6], fRY[2][6], fXG[2], fGR[2], fGU[2], fGCC[2], fGRH[2], fHG[2], fREF[2], fGG, fGC, fFBUF, fDY, fDY2,
      fDZc;
  DevBuf fGq, fGkk, fGv, fGnv, fGbb, fGsum, fdREF, fDZD, fDH, fDHA, fDRH, fDCP, fDGP, fDXG, fWT, fBN, fpart;
  // loss masks (cfg.mask_decoder): target lengths [B] on the device, their sum
  DevBuf TLEN;
  bool has_tlen = false;
  // style-embedding losses (cfg.n_emt / n_spk / orthog_weight): labels [2][B], the extra d refnet
  // outputs [2][B][128], classifier logit gradients [B][max(n)], the orthogonality product [B][B]
  DevBuf sLAB, sXREF, sDL, sOM;
  bool has_labels = false;
  long tlen_sum = 0;
  int tlen_max = 0;
  // teacher-forcing draw (tt2_train_set_teacher_forcing): feed[t] = 1 target frame t-1, 0 own frame
  std::vector<uint8_t> feed;
  // free-running steps: prenet-1 kernel transposed [P][NM], per-step scratch
  DevBuf W1T, sDZ, sDP, sDX;
  // persistent forward (train_persist.hip; TT2_TR_PERSIST=0 keeps the per-step launches): exchange
  // buffers, energy granules, flags + control words, the prenet rows in bf16 fragment layout
  DevBuf tpCX, tpH1X, tpZ1X, tpH2X, tpZ2X, tpEX, tpCtl, tpPre, tpStamps, tpKWT;
  bool tp_on = false, tp_last = false, tp_check = false;
  // persistent backward (train_bwd_persist.hip): exchange buffers, flags + control words
  DevBuf tbG1X, tbG2X, tbP1X, tbP2X, tbQX, tbCtl, tbW1F, tbPK, tbDGT1, tbDGT2, tbDGR1;
  DevBuf reg_segs;  // [nreg] (offset, size) of the regularised variables (tr_regularize)
  int nreg = 0;
  bool tb_dgt = false;  // the last persistent backward wrote bf16(dG)^T for the weight-gradient GEMMs
  bool tb_dgr = false;  // ... and bf16(dG1) row-major for the d X1 product
  bool tb_on = false, tb_last = false, tb_check = false;
  int* tb_ctl_dev = nullptr;
  int* tp_ctl_dev = nullptr;  // control words of the last persistent forward (device)
  int* tp_ctl_host = nullptr;  // pinned [2]: the launch's control words, checked at the next read-back
};

namespace tt2 {

constexpr int TR_MAX_TIN = 320;  // LDS budget of the attention kernels
constexpr int TR_JT = 16;        // j rows (encoder positions) per attention work-group
constexpr int TR_AT = 1024;      // threads of the energy / d-align / energy-backward work-groups

__device__ __forceinline__ float sigm_acc(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// block reductions (any multiple of 64 threads, <= 1024) through a 16-float LDS scratch
__device__ __forceinline__ float block_sum(float v, float* s16) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s16[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += s16[i];
  return r;
}
__device__ __forceinline__ float block_max(float v, float* s16) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s16[w] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, s16[i]);
  return r;
}

// ---- generic helpers ---------------------------------------------------------------------
// dst[c * ldd + r] = src[r * lds + c]  (32x32 LDS tiles)
__global__ __launch_bounds__(256) void k_tr_transpose(const float* __restrict__ src, long rows, long cols, long lds,
                                                      float* __restrict__ dst, long ldd) {
  __shared__ float tile[32][33];
  const long r0 = (long)blockIdx.y * 32, c0 = (long)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  for (int i = ty; i < 32; i += 8) {
    const long r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < rows && c < cols) ? src[r * lds + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const long c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[c * ldd + r] = tile[tx][i];
  }
}

// Column reductions over M rows of a row-major [M][N] matrix (column sums, BN statistics, BN
// backward sums) run as a (column tile, row split) grid: a tile is TW = 32 or 64 columns (32 when
// N < 64, so narrow matrices -- the reference encoders' 32-channel BN over ~10^6 positions -- keep
// every lane busy), the 256 threads of a work-group cover R = 256 / TW rows per pass, and the number
// of row splits S (tr_splits) fills the chip: ~2048 work-groups, at most TR_SMAX partials per column
// and at most `cap` partial floats (the partial buffers keep their sizes: 64 splits of the widest
// matrix each one serves, so narrow matrices get proportionally more splits).
constexpr int TR_SMAX = 512;
__host__ __device__ inline int tr_tw(int N) { return N < 64 ? 32 : 64; }
static inline int tr_splits(long M, int N, long cap) {
  const int tiles = (N + tr_tw(N) - 1) / tr_tw(N);
  const long rows_min = 64;  // >= 64 rows per split
  return (int)std::max<long>(1, std::min<long>({(long)TR_SMAX, 2048L / tiles, M / rows_min, cap / N}));
}

// partial column sums: part[s][n] = sum over rows m = s*R + r, + S*R, ... of in[m*ld + n]
__global__ __launch_bounds__(256) void k_tr_colsum_part(const float* __restrict__ in, long M, int N, long ld,
                                                        float* __restrict__ part) {
  __shared__ float red[256];
  const int TW = tr_tw(N), R = 256 / TW;
  const int c = threadIdx.x % TW, r = threadIdx.x / TW;
  const int n = blockIdx.x * TW + c;
  const int S = gridDim.y, s = blockIdx.y;
  float acc = 0.f;
  if (n < N) {
#pragma unroll 4
    for (long m = (long)s * R + r; m < M; m += (long)S * R) acc += in[m * ld + n];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (r == 0 && n < N) {
    float v = 0.f;
    for (int rr = 0; rr < R; ++rr) v += red[rr * TW + c];
    part[(long)s * N + n] = v;
  }
}
// Final pass of a split column reduction: Σ_s part[s·ld + n] for 32 columns per 1024-thread block
// (32 row groups x 8 independent accumulators: S = 512 partials are 2 rounds of loads, not 512
// dependent ones).  Valid on threads < 32 (row group 0); every thread must call it.
constexpr int TR_FIN = 1024;
__device__ __forceinline__ float colsum_fin(const float* __restrict__ part, int S, long ld, int n, bool ok,
                                            float* red /* [32][33] */) {
  const int c = threadIdx.x & 31, g = threadIdx.x >> 5;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ok)
    for (int s0 = g; s0 < S; s0 += 256) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int sp = s0 + 32 * u;
        if (sp < S) acc[u] += part[(long)sp * ld + n];
      }
    }
  red[g * 33 + c] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  float tot = 0.f;
  if (g == 0)
    for (int i = 0; i < 32; ++i) tot += red[i * 33 + c];
  __syncthreads();
  return tot;
}
__global__ __launch_bounds__(TR_FIN) void k_tr_colsum_final(const float* __restrict__ part, int S, int N,
                                                            float* __restrict__ out) {
  __shared__ float red[32 * 33];
  const int n = blockIdx.x * 32 + (threadIdx.x & 31);
  const float tot = colsum_fin(part, S, N, n, n < N, red);
  if (threadIdx.x < 32 && n < N) out[n] = tot;
}

__global__ void k_tr_to_bf16(const float* __restrict__ src, long n, __bf16* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (__bf16)src[i];
}

// ---- forward -------------------------------------------------------------------------------
// XIN[t][b] = t == 0 ? GO (zeros, helpers.py:136-138) : targets[b][t·r - 1], the last frame of step
// t-1's r (targets[:, r-1::r], helpers.py:78,126-129); targets [B][T·r][NM]
__global__ void k_tr_inputs(const float* __restrict__ tg, int B, int T, int NM, int r, float* __restrict__ xin) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)T * B * NM;
  if (i >= n) return;
  const int c = (int)(i % NM);
  const int b = (int)((i / NM) % B);
  const int t = (int)(i / ((long)NM * B));
  xin[i] = t == 0 ? 0.f : tg[((long)b * T * r + ((long)t * r - 1)) * NM + c];
}
// frame f of row b in the projection output [T][B][r·NM] (f = t·r + i -> row t·B + b, columns i·NM..)
__device__ __forceinline__ long tr_frame_off(int f, int b, int B, int r, int NM) {
  return (((long)(f / r) * B + b) * r + f % r) * NM;
}
// R > 1: dst[f][b][:] = FR frame (f, b): the clipped frames time-major for the Postnet's convolutions
__global__ void k_tr_frames_tm(const float* __restrict__ FR, int B, int Tf, int NM, int r, float* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Tf * B * NM) return;
  const int c = (int)(i % NM);
  const int b = (int)((i / NM) % B);
  const int f = (int)(i / ((long)NM * B));
  dst[i] = FR[tr_frame_off(f, b, B, r, NM) + c];
}
// values = memory · seq_mask (BahdanauAttention memory masking)
__global__ void k_tr_values(const float* __restrict__ mem, const int* __restrict__ lens, int B, int Tin, int D,
                            float* __restrict__ val) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * Tin * D) return;
  const int j = (int)((i / D) % Tin), b = (int)(i / ((long)D * Tin));
  val[i] = j < lens[b] ? mem[i] : 0.f;
}
// prenet dropout (modules.py:355, rate .5, always on): x = x / 0.5 · keep, in place on a strided
// [T·B, P] view; masks [T][2][B][P]
__global__ void k_tr_prenet_mask(float* __restrict__ x, long ld, const uint8_t* __restrict__ m, int layer, int T,
                                 int B, int P) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)T * B * P) return;
  const int p = (int)(i % P);
  const long tb = i / P;
  const int b = (int)(tb % B), t = (int)(tb / B);
  const float keep = (float)m[(((long)t * 2 + layer) * B + b) * P + p];
  x[tb * ld + p] = (x[tb * ld + p] / 0.5f) * keep;
}

// TF LSTMCell (modules.py:206) + training zoneout (modules.py:236-240) for one step.
// G [B,4H] pre-activations (bias added) -> overwritten with (σi, tanh j, σ(f+1), σo).
struct TrLstmFwd {
  float* G;
  const float* part;  // non-null: G's pre-activations = sum over ks raw split-K partials [ks][B][4H] + bias
  int ks;
  const float* bias;
  const float* c_prev;   // [B,H]
  const float* hz_prev;  // strided
  long ld_hz_prev;
  const uint8_t* zm;     // [T][4][B][H] or null (inference mix)
  int t, layer, B, H;
  float z;
  float* cn;       // [B,H] c_new
  float* c_out;    // [B,H] zoned c
  float* h_out;    // strided h_new
  long ld_h;
  float* hz_out;   // strided zoned h
  long ld_hz;
};
__global__ void k_tr_lstm_fwd(TrLstmFwd a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.B * a.H) return;
  const int b = i / a.H, n = i % a.H;
  float* g = a.G + (long)b * 4 * a.H;
  float pre[4];
  if (a.part) {  // fused split-K combine (gemm_raw): 4 independent chains, loads unrolled
#pragma unroll
    for (int q = 0; q < 4; ++q) pre[q] = a.bias[q * a.H + n];
    const float* p0 = a.part + (long)b * 4 * a.H + n;
    const long zs = (long)a.B * 4 * a.H;
#pragma unroll 4
    for (int z = 0; z < a.ks; ++z) {
      const float* pz = p0 + z * zs;
#pragma unroll
      for (int q = 0; q < 4; ++q) pre[q] += pz[q * a.H];
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) pre[q] = g[q * a.H + n];
  }
  const float si = sigm_acc(pre[0]), tj = tanhf(pre[1]), sf = sigm_acc(pre[2] + 1.0f), so = sigm_acc(pre[3]);
  g[n] = si;
  g[a.H + n] = tj;
  g[2 * a.H + n] = sf;
  g[3 * a.H + n] = so;
  const float cp = a.c_prev[i];
  const float hp = a.hz_prev[(long)b * a.ld_hz_prev + n];
  const float cnew = sf * cp + si * tj;
  const float hnew = so * tanhf(cnew);
  float c, h;
  if (a.zm) {
    const long base = (((long)a.t * 4 + 2 * a.layer) * a.B + b) * a.H + n;
    const float mc = (float)a.zm[base], mh = (float)a.zm[base + (long)a.B * a.H];
    c = cp + mc * (cnew - cp);
    h = hp + mh * (hnew - hp);
  } else {
    c = (1.f - a.z) * cnew + a.z * cp;
    h = (1.f - a.z) * hnew + a.z * hp;
  }
  a.cn[i] = cnew;
  a.c_out[i] = c;
  a.h_out[(long)b * a.ld_h + n] = hnew;
  a.hz_out[(long)b * a.ld_hz + n] = h;
}

// ---- fused skinny products of the decoder steps: bf16 product + epilogue in ONE launch ----------
// One decoder step's B <= 64-row products C = X·W (W as its pre-transposed bf16 copy Wt[N][K], so any
// column set is a set of contiguous K-vectors) with the consumer's epilogue fused, WHOLE K per
// work-group: no split-K partials and no combine launch.  Work-group = 32 output columns x one
// 32-row half; its 8 waves split K (K/8 each) and load their fragments 16 k-steps at a time
// (v_mfma_f32_32x32x16_bf16, one accumulator per wave); the 8 wave partials are summed in LDS.
// The two row halves of a column group are blocks g and g + 8, which share an XCD under
// round-robin dispatch, so the second read of the weight columns is an L2 hit (speed only).
//   TF_FWD   LSTM layer forward: columns {q·H + u0 + k} (q < 4 gates, k < 8 units), epilogue =
//            k_tr_lstm_fwd's cell + zoneout (Architecture_wrappers.py:214-224, zoneout_lstm.py)
//   TF_BWD_H LSTM layer-2 backward: columns = 32 units of d h (= d query · Wq^T, K = A, fp32 A
//            rows converted in-register) + d h from the frame projection, epilogue = k_tr_lstm_bwd's
//   TF_BWD_S LSTM layer-1 backward: columns = 16 units of d h1 and the same 16 of d hz2_{t-1}
//            (= dG2 · K2^T), the latter written out (+ R2), epilogue = k_tr_lstm_bwd's
//   TF_PLAIN C = X·W + residual (d X1 = dG1 · K1^T + R1)
// A operands are bf16 shadows of the fp32 rows written by their producers (same round-to-nearest-
// even as the staged operands of the bf16 GEMMs), except TF_BWD_H's.
enum { TF_FWD = 0, TF_BWD_H = 1, TF_BWD_S = 2, TF_PLAIN = 3, TF_EFWD = 4, TF_EBWD = 5 };
// Fragment-major bf16 layout of a [rows][K] operand ("TF layout"): 32-row blocks x 16-deep k-steps x
// [32 rows][16 k], so one wave's v_mfma_f32_32x32x16_bf16 fragment load of a k-step (lane l: row l%32,
// k = 8(l/32) .. +8) is ONE contiguous kilobyte instead of 32 rows a K-stride apart.  The weights are
// re-laid once per step in their column-group order (k_tr_tf_weights), the activation shadows are
// written in it by their producers; a step's row blocks cover Bp = B rounded up to 32 rows.
__host__ __device__ inline long tf_sw(int r, int k, int K) {
  return ((((long)(r >> 5) * (K >> 4) + (k >> 4)) * 32 + (r & 31)) << 4) + (k & 15);
}
__host__ __device__ inline long tf_colmap(int mode, int cg, int c, int H) {
  if (mode == TF_FWD || mode == TF_EFWD) return (long)(c >> 3) * H + cg * 8 + (c & 7);
  if (mode == TF_BWD_S) return c < 16 ? cg * 16 + c : H + cg * 16 + (c - 16);
  return (long)cg * 32 + c;
}
// W^T [N][K] bf16 -> TF layout in the fused kernel's column-group order (columns past N are zero)
__global__ void k_tr_tf_weights(const __bf16* __restrict__ src, int N, int K, int ncg, int mode, int H,
                                __bf16* __restrict__ dst) {
  const long n = (long)ncg * 32 * K;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / K), k = (int)(i % K);  // r = 32 cg + c
    const long col = tf_colmap(mode, r >> 5, r & 31, H);
    dst[tf_sw(r, k, K)] = col < N ? src[col * K + k] : (__bf16)0.f;
  }
}
// fp32 weights -> TF layout directly: element (column n, k) = src[n·ld + k], or src[k·ld + n] when
// transposed (the encoder LSTM's recurrent kernel serves both products: [U][4U] is W for the forward
// gates and W^T for the backward d h)
__global__ void k_tr_tf_weights_f32(const float* __restrict__ src, long ld, int transposed, int N, int K, int ncg,
                                    int mode, int H, __bf16* __restrict__ dst) {
  const long n = (long)ncg * 32 * K;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / K), k = (int)(i % K);
    const long col = tf_colmap(mode, r >> 5, r & 31, H);
    dst[tf_sw(r, k, K)] = col < N ? (__bf16)(transposed ? src[(long)k * ld + col] : src[col * ld + k]) : (__bf16)0.f;
  }
}
constexpr int TLG_U = 8, TLG_NT = 512, TLG_KSMAX = 16;
typedef float tlg_f32x16 __attribute__((ext_vector_type(16)));
struct TrFused {
  const __bf16* Ah;  // this step's bf16 input rows, TF layout of width K, or
  const float* Af;   // fp32 input rows (TF_BWD_H)
  long lda;
  int af_parts;      // > 1: each Af row is the sum of af_parts partial rows af_pstride apart (in order)
  int af_pstride;
  const __bf16* Wt;  // W^T in TF layout, column-group order (k_tr_tf_weights)
  int K, B, H, N;
  int t, layer;
  float z;
  const uint8_t* zm;     // [T][4][B][H] zoneout keep masks or null
  const float* G;        // fwd: out [B][4H] activated gates; bwd: in
  const float* bias;     // fwd
  const float* c_prev;   // [B,H]
  const float* hz_prev;  // fwd, strided
  long ld_hz_prev;
  float* cn;             // fwd out / bwd in [B,H]
  float* c_out;          // fwd [B,H]
  float* h_out;          // fwd strided h_new
  long ld_h;
  float* hz_out;         // fwd strided zoned h
  long ld_hz;
  __bf16* h_out_h;       // fwd bf16 TF-layout shadows (step block base, width ld_*_h, column offset
  long ld_h_h;           // *_col0) or null
  __bf16* hz_out_h;
  long ld_hz_h;
  int h_col0, hz_col0;
  const float* dh_ext;   // bwd: d h_new from the frame projection (strided) or null
  long ld_dh;
  float* side;           // TF_BWD_S: d hz2_{t-1} out (strided), = product + side_res[.][H + n]
  long ld_side;
  const float* side_res;
  long ld_side_res;
  const float* dhz;      // bwd: d(zoned h_t) from step t+1 (strided)
  long ld_dhz;
  float* DC;             // bwd [B,H] in/out
  float* dG;             // bwd out [B][4H]
  __bf16* dGh;           // bwd bf16 shadow of dG or null
  float* R;              // bwd [B][ldr] at off_r + n
  long ldr;
  int off_r;
  float* C;              // TF_PLAIN out (ld ldc) = product + residual
  long ldc;
  const float* residual;
  long ldres;
  // encoder BiLSTM (TF_EFWD / TF_EBWD, FeLstm's buffers; H = U, both directions in one launch)
  const int* lens;
  int T;                 // encoder steps
  float zo;
  long wdir, adir;       // per-direction strides of Wt and of the bf16 state shadow (elements)
  const float* XP;       // [B][T][8U] input projections (+ bias)
  float* GA; float* CN; float* CS; float* HS; float* ENC;
  __bf16* HSh;           // [2][T+1][Bp][U] TF layout: h state shadow (EFWD: A operand and output)
  const float* DENC; long ld_denc;
  float* DZ; float* DCC; float* DHP;
  __bf16* DZh;           // [2 dirs][2 slots][Bp][4U] TF layout: dZ shadow (EBWD: A of step t-1)
};

// Epilogue operands of one (row, unit), loaded BEFORE the product so their round trip overlaps the
// operand stream instead of following the reduction barrier.
struct TfCellIn {
  float g0, g1, g2, g3;  // fwd: bias of the 4 gates; bwd: the activated gates
  float cp, hp;          // c_{t-1}; fwd: zoned h_{t-1}
  float cn, dhz, dcz;    // bwd: c_new, d zoned h_t, d zoned c_t
  float ext, sres;       // bwd: d h_new from outside the product; TF_BWD_S: side residual
  float kc, kh;          // zoneout keep (mask) or 1 - z
};
template <int MODE>
__device__ __forceinline__ TfCellIn tf_cell_load(const TrFused& a, int b, int n) {
  TfCellIn v{};
  const long i = (long)b * a.H + n;
  if (a.zm) {
    const long base = (((long)a.t * 4 + 2 * a.layer) * a.B + b) * a.H + n;
    v.kc = (float)a.zm[base];
    v.kh = (float)a.zm[base + (long)a.B * a.H];
  } else {
    v.kc = v.kh = 1.f - a.z;
  }
  v.cp = a.c_prev[i];
  if constexpr (MODE == TF_FWD) {
    v.g0 = a.bias[n];
    v.g1 = a.bias[a.H + n];
    v.g2 = a.bias[2 * a.H + n];
    v.g3 = a.bias[3 * a.H + n];
    v.hp = a.hz_prev[(long)b * a.ld_hz_prev + n];
  } else {
    const float* g = a.G + (long)b * 4 * a.H;
    v.g0 = g[n];
    v.g1 = g[a.H + n];
    v.g2 = g[2 * a.H + n];
    v.g3 = g[3 * a.H + n];
    v.cn = a.cn[i];
    v.dhz = a.dhz[(long)b * a.ld_dhz + n];
    v.dcz = a.DC[i];
    v.ext = a.dh_ext ? a.dh_ext[(long)b * a.ld_dh + n] : 0.f;
    if constexpr (MODE == TF_BWD_S) v.sres = a.side_res[(long)b * a.ld_side_res + a.H + n];
  }
  return v;
}

// LSTM cell backward of one (row, unit) (k_tr_lstm_bwd): dext = d h_new from outside the cell
__device__ __forceinline__ void tf_cell_bwd(const TrFused& a, int b, int n, float dext, const TfCellIn& v) {
  const long i = (long)b * a.H + n;
  const float si = v.g0, tj = v.g1, sf = v.g2, so = v.g3;
  const float dhn = dext + v.kh * v.dhz;
  const float tc = tanhf(v.cn);
  const float dcn = v.kc * v.dcz + dhn * so * (1.f - tc * tc);
  const float dso = dhn * tc, dsf = dcn * v.cp, dsi = dcn * tj, dtj = dcn * si;
  const float d0 = dsi * si * (1.f - si), d1 = dtj * (1.f - tj * tj), d2 = dsf * sf * (1.f - sf), d3 = dso * so * (1.f - so);
  float* dg = a.dG + (long)b * 4 * a.H;
  dg[n] = d0;
  dg[a.H + n] = d1;
  dg[2 * a.H + n] = d2;
  dg[3 * a.H + n] = d3;
  if (a.dGh) {  // TF layout, width 4H
    const int K4 = 4 * a.H;
    a.dGh[tf_sw(b, n, K4)] = (__bf16)d0;
    a.dGh[tf_sw(b, a.H + n, K4)] = (__bf16)d1;
    a.dGh[tf_sw(b, 2 * a.H + n, K4)] = (__bf16)d2;
    a.dGh[tf_sw(b, 3 * a.H + n, K4)] = (__bf16)d3;
  }
  a.DC[i] = (1.f - v.kc) * v.dcz + dcn * sf;
  a.R[(long)b * a.ldr + a.off_r + n] = (1.f - v.kh) * v.dhz;
}

// Encoder BiLSTM cell of (direction, row, unit) at encoder step a.t (k_fe_lstm_cell /
// k_fe_lstm_cell_bwd of train_front.hip: TF's rnn step past a row's length copies the state and emits
// 0; the backward direction visits positions len-1-t), operands loaded before the product.
// TfCellIn: g0..g3 = input projections (fwd) / activated gates (bwd); cp, hp = c, h of step t (fwd)
// / c of step t (bwd); kc, kh = zoneout keep bits; dhz = d h_t from the output (bwd), dcz = d carried
// c, ext = the carried d h's direct part (DHP) of step t+1, cn = c_new (bwd), sres = the row's length
template <int MODE>
__device__ __forceinline__ TfCellIn tf_enc_load(const TrFused& a, int dir, int b, int u) {
  TfCellIn v{};
  const int U = a.H, B = a.B, T = a.T, t = a.t;
  const int len = a.lens[b];
  v.sres = (float)len;
  if (a.zm) {
    v.kc = (float)a.zm[((((long)t * 2 + dir) * 2 + 0) * B + b) * U + u];
    v.kh = (float)a.zm[((((long)t * 2 + dir) * 2 + 1) * B + b) * U + u];
  } else {
    v.kc = v.kh = 1.f - a.zo;
  }
  const long st0 = ((long)dir * (T + 1) + t) * B * U + (long)b * U + u;
  const int pos = dir == 0 ? t : len - 1 - t;
  if constexpr (MODE == TF_EFWD) {
    v.cp = a.CS[st0];
    v.hp = a.HS[st0];
    if (t < len) {
      const float* xp = a.XP + ((long)b * T + pos) * 8 * U + dir * 4 * U;
      v.g0 = xp[u];
      v.g1 = xp[U + u];
      v.g2 = xp[2 * U + u];
      v.g3 = xp[3 * U + u];
    }
  } else {
    const long sidx = ((long)dir * B + b) * U + u;
    v.ext = a.DHP[sidx];
    v.dcz = a.DCC[sidx];
    if (t < len) {
      const float* ga = a.GA + (((long)dir * T + t) * B + b) * 4 * U;
      v.g0 = ga[u];
      v.g1 = ga[U + u];
      v.g2 = ga[2 * U + u];
      v.g3 = ga[3 * U + u];
      v.cn = a.CN[((long)dir * T + t) * B * U + (long)b * U + u];
      v.cp = a.CS[st0];
      v.dhz = a.DENC[((long)b * T + pos) * a.ld_denc + dir * U + u];
    }
  }
  return v;
}
__device__ __forceinline__ void tf_enc_fwd(const TrFused& a, int dir, int b, int u, float p0, float p1, float p2, float p3,
                                           const TfCellIn& v) {
  const int U = a.H, B = a.B, T = a.T, t = a.t, len = (int)v.sres;
  const long st1 = ((long)dir * (T + 1) + t + 1) * B * U + (long)b * U + u;
  const int Bp = (B + 31) & ~31;
  __bf16* hs1 = a.HSh + dir * a.adir + (long)(t + 1) * Bp * U;
  if (t >= len) {  // past the row's length: state copied, output stays 0 (TF rnn._rnn_step)
    a.CS[st1] = v.cp;
    a.HS[st1] = v.hp;
    hs1[tf_sw(b, u, U)] = (__bf16)v.hp;
    return;
  }
  const int pos = dir == 0 ? t : len - 1 - t;
  const float si = 1.0f / (1.0f + expf(-(p0 + v.g0))), tj = tanhf(p1 + v.g1);
  const float sf = 1.0f / (1.0f + expf(-(p2 + v.g2 + 1.0f))), so = 1.0f / (1.0f + expf(-(p3 + v.g3)));
  const float cn = sf * v.cp + si * tj;
  const float hn = so * tanhf(cn);
  float* ga = a.GA + (((long)dir * T + t) * B + b) * 4 * U;
  ga[u] = si;
  ga[U + u] = tj;
  ga[2 * U + u] = sf;
  ga[3 * U + u] = so;
  a.CN[((long)dir * T + t) * B * U + (long)b * U + u] = cn;
  const float hs = v.hp + v.kh * (hn - v.hp);
  a.CS[st1] = v.cp + v.kc * (cn - v.cp);
  a.HS[st1] = hs;
  hs1[tf_sw(b, u, U)] = (__bf16)hs;
  a.ENC[((long)b * T + pos) * 2 * U + dir * U + u] = hn;
}
__device__ __forceinline__ void tf_enc_bwd(const TrFused& a, int dir, int b, int u, float prod, const TfCellIn& v) {
  const int U = a.H, B = a.B, T = a.T, t = a.t, len = (int)v.sres;
  const long sidx = ((long)dir * B + b) * U + u;
  const int Bp = (B + 31) & ~31;
  const float dhc = prod + v.ext;  // d h carried out of step t = dZ(t+1)·Wh^T + its direct part
  float* dz = a.DZ + (((long)dir * T + t) * B + b) * 4 * U;
  __bf16* dzh = a.DZh + dir * a.adir + (long)(t & 1) * Bp * 4 * U;
  if (t >= len) {  // copied state: gradients pass through, no gate gradient
    dz[u] = dz[U + u] = dz[2 * U + u] = dz[3 * U + u] = 0.f;
    dzh[tf_sw(b, u, 4 * U)] = dzh[tf_sw(b, U + u, 4 * U)] = dzh[tf_sw(b, 2 * U + u, 4 * U)] =
        dzh[tf_sw(b, 3 * U + u, 4 * U)] = (__bf16)0.f;
    a.DHP[sidx] = dhc;
    return;
  }
  const float si = v.g0, tj = v.g1, sf = v.g2, so = v.g3;
  const float dhn = v.dhz + v.kh * dhc;
  const float tc = tanhf(v.cn);
  const float dcn = v.kc * v.dcz + dhn * so * (1.f - tc * tc);
  const float d0 = dcn * tj * si * (1.f - si), d1 = dcn * si * (1.f - tj * tj);
  const float d2 = dcn * v.cp * sf * (1.f - sf), d3 = dhn * tc * so * (1.f - so);
  dz[u] = d0;
  dz[U + u] = d1;
  dz[2 * U + u] = d2;
  dz[3 * U + u] = d3;
  dzh[tf_sw(b, u, 4 * U)] = (__bf16)d0;
  dzh[tf_sw(b, U + u, 4 * U)] = (__bf16)d1;
  dzh[tf_sw(b, 2 * U + u, 4 * U)] = (__bf16)d2;
  dzh[tf_sw(b, 3 * U + u, 4 * U)] = (__bf16)d3;
  a.DCC[sidx] = (1.f - v.kc) * v.dcz + dcn * sf;
  a.DHP[sidx] = (1.f - v.kh) * dhc;
}

template <int MODE>
__global__ __launch_bounds__(TLG_NT, 1) void k_tr_fused(TrFused a) {
  typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
  __shared__ float red[8][32][33];  // wave partials [w][row][col] (padded)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ncg = gridDim.x >> 1, bid = blockIdx.x;
  const int cg = (ncg & 7) == 0 ? (bid & 7) + 8 * (bid >> 4) : bid >> 1;
  const int rh = (ncg & 7) == 0 ? (bid >> 3) & 1 : bid & 1;
  const int r0 = 32 * rh;
  // encoder modes: the column groups of direction 1 follow those of direction 0
  constexpr bool ENC = MODE == TF_EFWD || MODE == TF_EBWD;
  const int dir = ENC ? cg / (ncg >> 1) : 0, cgl = ENC ? cg % (ncg >> 1) : cg;
  const __bf16* const Wb = a.Wt + (ENC ? dir * a.wdir : 0L);
  const int Bp = (a.B + 31) & ~31;
  const __bf16* const Ab = MODE == TF_EFWD ? a.HSh + dir * a.adir + (long)a.t * Bp * a.H
                           : MODE == TF_EBWD ? a.DZh + dir * a.adir + (long)((a.t + 1) & 1) * Bp * 4 * a.H
                                             : a.Ah;
  // this thread's epilogue element(s): FWD / EFWD 32 rows x 8 units (threads < 256), BWD_S 32 x 16,
  // BWD_H / EBWD 32 x 32 units and PLAIN 32 x 32 columns (two per thread)
  constexpr int NE = (MODE == TF_BWD_H || MODE == TF_PLAIN || MODE == TF_EBWD) ? 2 : 1;
  constexpr int UPR = (MODE == TF_FWD || MODE == TF_EFWD) ? 8 : MODE == TF_BWD_S ? 16 : 32;  // columns per row
  int eb[NE], en[NE], erl[NE], ekk[NE];
  bool eok[NE];
  TfCellIn ev[NE];
  float eres[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int pidx = tid + TLG_NT * e;
    erl[e] = pidx / UPR;
    ekk[e] = pidx % UPR;
    eb[e] = r0 + erl[e];
    en[e] = cgl * UPR + ekk[e];
    eok[e] = erl[e] < 32 && eb[e] < a.B && (MODE != TF_PLAIN || en[e] < a.N);
    eres[e] = 0.f;
    if constexpr (MODE == TF_PLAIN) {
      if (eok[e] && a.residual) eres[e] = a.residual[(long)eb[e] * a.ldres + en[e]];
    } else if constexpr (ENC) {
      if (eok[e]) ev[e] = tf_enc_load<MODE>(a, dir, eb[e], en[e]);
    } else {
      if (eok[e]) ev[e] = tf_cell_load<MODE>(a, eb[e], en[e]);
    }
  }
  const int kw = a.K >> 3, k0 = w * kw, ks = kw >> 4;  // host: K % 128 == 0
  const int c = lane & 31, kh = 8 * (lane >> 5);
  const bool rok = r0 + c < a.B;
  const bf8 z8 = {};
  tlg_f32x16 acc = {};
  if (MODE != TF_BWD_H && ks == 2 * TLG_KSMAX) {
    // K = 4096 (the LSTM backward products, d X1): a rolling pipeline over the wave's 32 k-steps, fully
    // unrolled and branch-free (rows past B load row 0 and are zeroed by a select; the second row half
    // of a B <= 32 launch lies past the Bp-row shadow),
    // so the slot a k-step's MFMA frees is refilled with the k-step 16 ahead while the first loads
    // are still landing: the K range costs one memory round trip instead of two batches back to back
    bf8 va[TLG_KSMAX], vb[TLG_KSMAX];
    const __bf16* const wrow = Wb + tf_sw(32 * cgl + c, k0 + kh, a.K);
    const __bf16* const arow = Ab + tf_sw(rok ? r0 + c : 0, k0 + kh, a.K);  // row 0: always allocated
    // tf_sw(r, k + 16 j, K) = tf_sw(r, k, K) + 512 j for k % 16 == kh (16-deep k-steps of 32 x 16)
#pragma unroll
    for (int s = 0; s < TLG_KSMAX; ++s) {
      vb[s] = *reinterpret_cast<const bf8*>(wrow + 512 * s);
      const bf8 x = *reinterpret_cast<const bf8*>(arow + 512 * s);
      va[s] = rok ? x : z8;
    }
#pragma unroll
    for (int ss = 0; ss < 2 * TLG_KSMAX; ++ss) {
      const int s = ss % TLG_KSMAX;
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[s], vb[s], acc, 0, 0, 0);
      if (ss + TLG_KSMAX < 2 * TLG_KSMAX) {
        vb[s] = *reinterpret_cast<const bf8*>(wrow + 512 * (ss + TLG_KSMAX));
        const bf8 x = *reinterpret_cast<const bf8*>(arow + 512 * (ss + TLG_KSMAX));
        va[s] = rok ? x : z8;
      }
    }
  } else
  for (int s0 = 0; s0 < ks; s0 += TLG_KSMAX) {
    bf8 va[TLG_KSMAX], vb[TLG_KSMAX];
#pragma unroll
    for (int s = 0; s < TLG_KSMAX; ++s) {
      if (s0 + s < ks) {
        const int k = k0 + 16 * (s0 + s) + kh;
        vb[s] = *reinterpret_cast<const bf8*>(Wb + tf_sw(32 * cgl + c, k, a.K));
        if constexpr (MODE == TF_BWD_H) {
          if (rok) {
            const float* p = a.Af + (long)(r0 + c) * a.lda + k;
            f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
            for (int g = 1; g < a.af_parts; ++g) {
              x0 += *reinterpret_cast<const f32x4*>(p + (long)g * a.af_pstride);
              x1 += *reinterpret_cast<const f32x4*>(p + (long)g * a.af_pstride + 4);
            }
            va[s] = bf8{(__bf16)x0[0], (__bf16)x0[1], (__bf16)x0[2], (__bf16)x0[3],
                        (__bf16)x1[0], (__bf16)x1[1], (__bf16)x1[2], (__bf16)x1[3]};
          } else {
            va[s] = z8;
          }
        } else {
          va[s] = rok ? *reinterpret_cast<const bf8*>(Ab + tf_sw(r0 + c, k, a.K)) : z8;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < TLG_KSMAX; ++s)
      if (s0 + s < ks) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[s], vb[s], acc, 0, 0, 0);
  }
  // D layout: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][(r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)][c] = acc[r];
  __syncthreads();
  const auto sum8 = [&](int rl, int cc) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) v += red[ww][rl][cc];
    return v;
  };
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    if (!eok[e]) continue;
    const int rl = erl[e], kk = ekk[e], b = eb[e], n = en[e];
    if constexpr (MODE == TF_FWD) {
      const TfCellIn& v = ev[e];
      const float pre0 = v.g0 + sum8(rl, kk), pre1 = v.g1 + sum8(rl, 8 + kk);
      const float pre2 = v.g2 + sum8(rl, 16 + kk), pre3 = v.g3 + sum8(rl, 24 + kk);
      const float si = sigm_acc(pre0), tj = tanhf(pre1), sf = sigm_acc(pre2 + 1.0f), so = sigm_acc(pre3);
      float* g = const_cast<float*>(a.G) + (long)b * 4 * a.H;
      g[n] = si;
      g[a.H + n] = tj;
      g[2 * a.H + n] = sf;
      g[3 * a.H + n] = so;
      const long i = (long)b * a.H + n;
      const float cnew = sf * v.cp + si * tj;
      const float hnew = so * tanhf(cnew);
      float cz, hz;
      if (a.zm) {
        cz = v.cp + v.kc * (cnew - v.cp);
        hz = v.hp + v.kh * (hnew - v.hp);
      } else {
        cz = (1.f - a.z) * cnew + a.z * v.cp;
        hz = (1.f - a.z) * hnew + a.z * v.hp;
      }
      a.cn[i] = cnew;
      a.c_out[i] = cz;
      a.h_out[(long)b * a.ld_h + n] = hnew;
      a.hz_out[(long)b * a.ld_hz + n] = hz;
      if (a.h_out_h) a.h_out_h[tf_sw(b, a.h_col0 + n, (int)a.ld_h_h)] = (__bf16)hnew;
      if (a.hz_out_h) a.hz_out_h[tf_sw(b, a.hz_col0 + n, (int)a.ld_hz_h)] = (__bf16)hz;
    } else if constexpr (MODE == TF_EFWD) {
      tf_enc_fwd(a, dir, b, n, sum8(rl, kk), sum8(rl, 8 + kk), sum8(rl, 16 + kk), sum8(rl, 24 + kk), ev[e]);
    } else if constexpr (MODE == TF_EBWD) {
      tf_enc_bwd(a, dir, b, n, sum8(rl, kk), ev[e]);
    } else if constexpr (MODE == TF_BWD_H) {
      tf_cell_bwd(a, b, n, sum8(rl, kk) + ev[e].ext, ev[e]);
    } else if constexpr (MODE == TF_BWD_S) {
      a.side[(long)b * a.ld_side + n] = sum8(rl, 16 + kk) + ev[e].sres;
      tf_cell_bwd(a, b, n, sum8(rl, kk), ev[e]);
    } else {
      a.C[(long)b * a.ldc + n] = sum8(rl, kk) + eres[e];
    }
  }
}

// dst[r][c] = src[r][c] (+ add[r][c]): strided row-block copies (use_gst = 0 style embeddings)
__global__ void k_tr_rows_copy(const float* __restrict__ src, long lds, long rows, int cols, float* __restrict__ dst,
                               long ldd, const float* __restrict__ add, long ldadd) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const long r = i / cols, cc = i % cols;
  dst[r * ldd + cc] = src[r * lds + cc] + (add ? add[r * ldadd + cc] : 0.f);
}

// fp32 rows [rows][cols] (ld lds; row r = step r / B, row r % B) -> the bf16 TF-layout shadow of width
// K (steps of Bp rows): the fused products' input rows that no kernel writes as a by-product (prenet)
__global__ void k_tr_rows_bf16(const float* __restrict__ src, long lds, long rows, int cols, int B, int K,
                               __bf16* __restrict__ dst) {
  const long n = rows * cols;
  const long Bp = (B + 31) & ~31;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols, cc = i % cols;
    dst[(r / B) * Bp * K + tf_sw((int)(r % B), (int)cc, K)] = (__bf16)src[r * lds + cc];
  }
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
struct TrAtt {
  int B, Tin, T, A, F, KW, D, H, P, t, nt;  // nt = j-tiles per row (TR_JT rows each)
  int smooth;           // hp.smoothing: a = sigmoid(e) / Σ sigmoid(e) (attention.py:71-91) instead of softmax
  float* SS;            // [T][B] Σ_j sigmoid(e_j) of each step (smooth): sigmoid(e_j) = a_j·SS for the backward
  const int* lens;
  const float* keys;    // [B,Tin,A]
  const float* values;  // [B,Tin,D]
  const __bf16* values16;  // non-null (bf16 step): the same values rounded to bf16, read by the context
                           // product (half the bytes of its dominant read)
  const float* Q;       // [T][B][A]
  const float* qpart;   // non-null: the step's query as raw split-K partials [qks][B][A] (k_tr_att_energy2
  int qks;              // sums them: no combine launch), else Q
  const float* Kc;      // [KW][F] location conv kernel
  const float* bc;      // [F]
  const float* Wl;      // [F][A]
  const float* va;      // [A]
  const float* ba;      // [A]
  float* ALIGN;         // [B][Tin][T]
  float* CUM;           // [(T+1)][B][Tin]
  float* TH;            // [T][B][Tin][A] tanh(keys + q + loc + b_a); the backward overwrites it with du
  float* FALL;          // [T][B][Tin][F] location features (for d W_loc = Σ f^T du after the loop)
  float* ALN;           // [T][B][Tin] alignments, time-major copy for coalesced backward reads
  float* E;             // [B][Tin] energies of the current step
  // forward outputs of the context
  float* PIN;
  float* X1;
  __bf16* X1h;  // bf16 shadow of X1 (fused LSTM products) or null
  // backward
  const float* dPIN;
  const float* dX1;
  float* DF;     // [B][Tin][F] d location features
  float* PQ;     // [B][nt][A] per-tile d query partials
  float* DCTX;   // [T][B][D]
  float* DQ;     // [T][B][A]
  float* DKEYS;  // [B][Tin][A]
  float* DCUM;   // [B][Tin]
  float* dV;     // [B][nt][A]   accumulated over steps
  float* dBA;    // [B][nt][A]
  float* dKC;    // [B][nt][KW][F]
  float* dBC;    // [B][nt][F]
  long long* stamps;  // diagnostic: k_tr_att_bwd_q stage stamps of step stamp_t ([B][4][16]) or null
  int stamp_t;
  float* DWGP;   // [B][nt][32][A] k_tr_att_bwd_q: Σ_t G[tap][a] = Σ_j cum_{t-1}[j + tap - pad]·du[j][a] (d W_loc)
};

// Location features of rows j0..j0+TR_JT-1 of utterance b (attention.py:193-195):
// f[jj][c] = bc[c] + Σ_tap cum_{t-1}[j0 + jj + tap - pad]·Kc[tap][c]; cseg = the cum segment.
__device__ __forceinline__ void tr_locf_tile(const TrAtt& a, int b, int j0, float* cseg, float* f, float* Kcs) {
  const int pad = (a.KW - 1) / 2;
  const float* cum_prev = a.CUM + ((long)a.t * a.B + b) * a.Tin;
  for (int i = threadIdx.x; i < TR_JT + a.KW - 1; i += blockDim.x) {
    const int j = j0 + i - pad;
    cseg[i] = (j >= 0 && j < a.Tin) ? cum_prev[j] : 0.f;
  }
  for (int i = threadIdx.x; i < a.KW * a.F; i += blockDim.x) Kcs[i] = a.Kc[i];  // taps from LDS
  __syncthreads();
  for (int i = threadIdx.x; i < TR_JT * a.F; i += blockDim.x) {
    const int jj = i / a.F, c = i % a.F;
    float acc = a.bc[c];
    for (int tap = 0; tap < a.KW; ++tap) acc += cseg[jj + tap] * Kcs[tap * a.F + c];
    f[i] = acc;
  }
  __syncthreads();
}

// Energies e_j = Σ_k v_a[k]·tanh(keys_jk + q_k + loc_jk + b_a[k]) (attention.py:37-69) for one
// tile of TR_JT rows; grid (nt, B) spreads a step over the chip.  Keeps tanh for the backward.
__global__ __launch_bounds__(TR_AT) void k_tr_att_energy(TrAtt a) {
  __shared__ float cseg[TR_JT + 64];
  __shared__ float f[TR_JT * 32];
  __shared__ float Wl[32 * 256];
  __shared__ float Kcs[65 * 32];  // attention_kernel <= 65, attention_filters <= 32 (tt2_train_create)
  const int b = blockIdx.y, j0 = blockIdx.x * TR_JT;
  for (int i = threadIdx.x; i < a.F * a.A; i += blockDim.x) Wl[i] = a.Wl[i];
  tr_locf_tile(a, b, j0, cseg, f, Kcs);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const long tb = (long)a.t * a.B + b;
  for (int i = threadIdx.x; i < TR_JT * a.F; i += blockDim.x) {
    const int j = j0 + i / a.F;
    if (j < a.Tin) a.FALL[(tb * a.Tin + j0) * a.F + i] = f[i];
  }
  const float* q = a.Q + tb * a.A;
  for (int jj = wave; jj < TR_JT; jj += nw) {
    const int j = j0 + jj;
    if (j >= a.Tin) break;
    float acc = 0.f;
    for (int k = lane; k < a.A; k += 64) {
      float u = a.keys[((long)b * a.Tin + j) * a.A + k] + q[k] + a.ba[k];
      for (int c = 0; c < a.F; ++c) u += f[jj * a.F + c] * Wl[c * a.A + k];
      const float th = tanhf(u);
      a.TH[(tb * a.Tin + j) * a.A + k] = th;
      acc += a.va[k] * th;
    }
    acc = wave_sum(acc);
    if (lane == 0) a.E[(long)b * a.Tin + j] = acc;
  }
}

// Same energies with 256 threads (A <= 128): the lane's two W_loc columns live in registers (64
// VGPRs, loaded once from L2), so a row costs 8 broadcast 16-byte LDS reads of its location features
// instead of 64 LDS reads per column pair; the wave's 4 rows have their keys prefetched with the
// staging loads.  Four 256-thread work-groups fit a CU where one 1024-thread one did: the (j-tile,
// row) grid runs in one wave of work-groups.
constexpr int TR_E2T = 256;
__global__ __launch_bounds__(TR_E2T) void k_tr_att_energy2(TrAtt a) {
  __shared__ float cseg[TR_JT + 64];
  __shared__ __attribute__((aligned(16))) float f[TR_JT * 32];
  __shared__ float Kcs[65 * 32];
  const int b = blockIdx.y, j0 = blockIdx.x * TR_JT, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int F = a.F, A = a.A, Tin = a.Tin, pad = (a.KW - 1) / 2;
  const long tb = (long)a.t * a.B + b;
  const int k0 = lane, k1 = lane + 64;
  const bool ok0 = k0 < A, ok1 = k1 < A;
  float wl0[32], wl1[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    wl0[c] = (c < F && ok0) ? a.Wl[c * A + k0] : 0.f;
    wl1[c] = (c < F && ok1) ? a.Wl[c * A + k1] : 0.f;
  }
  float key0[4], key1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = j0 + w + 4 * r;
    const bool jok = j < Tin;
    key0[r] = (jok && ok0) ? a.keys[((long)b * Tin + j) * A + k0] : 0.f;
    key1[r] = (jok && ok1) ? a.keys[((long)b * Tin + j) * A + k1] : 0.f;
  }
  float q0 = 0.f, q1 = 0.f;
  if (a.qpart) {  // fused split-K combine of the query product (partials in split order; up to 16
                  // splits loaded in one round trip, before any sum)
    const float* qp = a.qpart + (long)b * A;
    const long zs = (long)a.B * A;
    if (a.qks <= 16) {
      float p0[16], p1[16];
#pragma unroll
      for (int z = 0; z < 16; ++z) {
        p0[z] = (z < a.qks && ok0) ? qp[z * zs + k0] : 0.f;
        p1[z] = (z < a.qks && ok1) ? qp[z * zs + k1] : 0.f;
      }
#pragma unroll
      for (int z = 0; z < 16; ++z) {
        q0 += p0[z];
        q1 += p1[z];
      }
    } else {
      for (int z = 0; z < a.qks; ++z) {
        if (ok0) q0 += qp[z * zs + k0];
        if (ok1) q1 += qp[z * zs + k1];
      }
    }
  } else {
    const float* q = a.Q + tb * A;
    q0 = ok0 ? q[k0] : 0.f;
    q1 = ok1 ? q[k1] : 0.f;
  }
  const float qb0 = ok0 ? q0 + a.ba[k0] : 0.f, qb1 = ok1 ? q1 + a.ba[k1] : 0.f;
  const float va0 = ok0 ? a.va[k0] : 0.f, va1 = ok1 ? a.va[k1] : 0.f;
  const float* cum_prev = a.CUM + tb * Tin;
  for (int i = tid; i < TR_JT + a.KW - 1; i += TR_E2T) {
    const int j = j0 + i - pad;
    cseg[i] = (j >= 0 && j < Tin) ? cum_prev[j] : 0.f;
  }
  for (int i = tid; i < a.KW * F; i += TR_E2T) Kcs[i] = a.Kc[i];
  __syncthreads();
  for (int i = tid; i < TR_JT * 32; i += TR_E2T) {  // location features (attention.py:193-195)
    const int jj = i >> 5, c = i & 31;
    float acc = 0.f;
    if (c < F) {
      acc = a.bc[c];
      for (int tap = 0; tap < a.KW; ++tap) acc += cseg[jj + tap] * Kcs[tap * F + c];
      if (j0 + jj < Tin) a.FALL[(tb * Tin + j0 + jj) * F + c] = acc;
    }
    f[i] = acc;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int jj = w + 4 * r, j = j0 + jj;
    if (j >= Tin) break;
    const f32x4* fr = reinterpret_cast<const f32x4*>(f + jj * 32);
    float u0 = key0[r] + qb0, u1 = key1[r] + qb1;
#pragma unroll
    for (int c4 = 0; c4 < 8; ++c4) {
      const f32x4 fv = fr[c4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        u0 += fv[e] * wl0[4 * c4 + e];
        u1 += fv[e] * wl1[4 * c4 + e];
      }
    }
    float acc = 0.f;
    const long hrow = (tb * Tin + j) * A;
    if (ok0) {
      const float th = tanhf(u0);
      a.TH[hrow + k0] = th;
      acc += va0 * th;
    }
    if (ok1) {
      const float th = tanhf(u1);
      a.TH[hrow + k1] = th;
      acc += va1 * th;
    }
    acc = wave_sum(acc);
    if (lane == 0) a.E[(long)b * Tin + j] = acc;
  }
}

// Masked softmax (attention.py:218, TF _maybe_mask_score) recomputed by every block of the row,
// cumulative alignments (:222-225) by block 0, then context_t = align_t · values (:27)
// -> PIN[t][b][H:], X1[t+1][b][P:P+D].
__global__ __launch_bounds__(256) void k_tr_ctx(TrAtt a) {
  extern __shared__ float al[];
  __shared__ float s16[16];
  const int b = blockIdx.y;
  const int len = a.lens[b];
  const float* e = a.E + (long)b * a.Tin;
  float mx = -INFINITY;
  if (!a.smooth) {
    for (int j = threadIdx.x; j < len; j += blockDim.x) mx = fmaxf(mx, e[j]);
    mx = block_max(mx, s16);
  }
  float sm = 0.f;
  for (int j = threadIdx.x; j < a.Tin; j += blockDim.x) {
    // masked positions score -inf: exp -> 0, and sigmoid(-inf) = 0 under the smoothing normalisation
    const float x = j < len ? (a.smooth ? 1.f / (1.f + expf(-e[j])) : expf(e[j] - mx)) : 0.f;
    al[j] = x;
    sm += x;
  }
  sm = block_sum(sm, s16);
  const long tb = (long)a.t * a.B + b;
  if (a.smooth && blockIdx.x == 0 && threadIdx.x == 0) a.SS[tb] = sm;
  for (int j = threadIdx.x; j < a.Tin; j += blockDim.x) {
    const float x = al[j] / sm;
    al[j] = x;
    if (blockIdx.x == 0) {
      a.ALIGN[((long)b * a.Tin + j) * a.T + a.t] = x;
      a.ALN[tb * a.Tin + j] = x;
      a.CUM[(tb + a.B) * a.Tin + j] = a.CUM[tb * a.Tin + j] + x;
    }
  }
  __syncthreads();
  // 64 channels per work-group.  D % 4 == 0: 16 float4 columns x 16 row groups, every row of a batch
  // of 10 loaded before its products (the values rows are the kernel's whole read); else 4 row groups
  __shared__ float red[16][64];
  const int tid = threadIdx.x;
  if ((a.D & 3) == 0) {
    const int cg = tid & 15, rg = tid >> 4, nc0 = blockIdx.x * 64 + 4 * cg;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (nc0 < a.D) {
      const float* vb = a.values + (long)b * a.Tin * a.D + nc0;
      const __bf16* vb16 = a.values16 ? a.values16 + (long)b * a.Tin * a.D + nc0 : nullptr;
      for (int j0 = rg; j0 < a.Tin; j0 += 160) {
        f32x4 v[10];
        if (vb16) {
#pragma unroll
          for (int u = 0; u < 10; ++u) {
            const int j = j0 + 16 * u;
            bf16x4 h = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
            if (j < a.Tin) h = *reinterpret_cast<const bf16x4*>(vb16 + (long)j * a.D);
            v[u] = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
          }
        } else {
#pragma unroll
          for (int u = 0; u < 10; ++u) {
            const int j = j0 + 16 * u;
            v[u] = j < a.Tin ? *reinterpret_cast<const f32x4*>(vb + (long)j * a.D) : f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
#pragma unroll
        for (int u = 0; u < 10; ++u) {
          const int j = j0 + 16 * u;
          if (j < a.Tin) acc += al[j] * v[u];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[rg][4 * cg + i] = acc[i];
    __syncthreads();
    const int nc = blockIdx.x * 64 + tid;
    if (tid < 64 && nc < a.D) {
      float r = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) r += red[g][tid];
      a.PIN[tb * (a.H + a.D) + a.H + nc] = r;
      a.X1[(tb + a.B) * (a.P + a.D + a.H) + a.P + nc] = r;
      if (a.X1h) {  // TF layout, step block t+1 of Bp rows
        const int LX = a.P + a.D + a.H, Bp = (a.B + 31) & ~31;
        a.X1h[(long)(a.t + 1) * Bp * LX + tf_sw(b, a.P + nc, LX)] = (__bf16)r;
      }
    }
    return;
  }
  const int nl = tid & 63, wq = tid >> 6;
  const int nc = blockIdx.x * 64 + nl;
  float acc = 0.f;
  if (nc < a.D) {
    const float* v = a.values + (long)b * a.Tin * a.D + nc;
#pragma unroll 4
    for (int j = wq; j < a.Tin; j += 4) acc += al[j] * v[(long)j * a.D];
  }
  red[wq][nl] = acc;
  __syncthreads();
  if (wq == 0 && nc < a.D) {
    const float r = red[0][nl] + red[1][nl] + red[2][nl] + red[3][nl];
    a.PIN[tb * (a.H + a.D) + a.H + nc] = r;
    a.X1[(tb + a.B) * (a.P + a.D + a.H) + a.P + nc] = r;
  }
}

// frame MSE + stop sigmoid CE (tacotron.py:774,778-779) and their output gradients.  Frames are
// time-major [T][B][NM]; targets [B][T][NM].  Deterministic per-block partials.
// tlen (mask_decoder, tacotron.py:758-767): MaskedMSE = Σ w·d² / (NM·Σ lengths) (the count of nonzero
// weights, tf.losses SUM_BY_NONZERO_WEIGHTS), MaskedSigmoidCrossEntropy = Σ w·wce / count_nonzero(w·wce)
// with TF's weighted_cross_entropy_with_logits (pos_weight q): (1-z)x + (1+(q-1)z)·softplus(-x)
// (modules.py:532-575).  The masked stop gradient is left unnormalised (the count is only known after
// the reduction; k_tr_loss_final / k_tr_div finish it).  inv_f = 1 / (MSE normaliser).
__global__ __launch_bounds__(256) void k_tr_loss(float* __restrict__ FR, const float* __restrict__ ST,
                                                 const float* __restrict__ tg, const float* __restrict__ stg, int B,
                                                 int T, int NM, int r, int clip, float lo, float hi,
                                                 float* __restrict__ dFR,
                                                 float* __restrict__ dST, float* __restrict__ part,
                                                 uint8_t* __restrict__ clipm, const int* __restrict__ tlen, float inv_f,
                                                 float pos_weight) {
  __shared__ float s4[16];
  // T = frames here (decoder steps · r); frame (t, b) of FR / dFR / clipm at tr_frame_off, stop (t, b)
  // of ST / dST at [t / r][b][t % r] (the r-wide stop projection; r = 1: [t][b])
  const long nf = (long)T * B * NM;
  const float inv_s = 1.0f / (float)((long)T * B);
  float sq = 0.f, ce = 0.f, nz = 0.f;
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < nf; i0 += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i0 % NM);
    const int b = (int)((i0 / NM) % B);
    const int t = (int)(i0 / ((long)NM * B));
    const long i = r == 1 ? i0 : tr_frame_off(t, b, B, r, NM) + c;
    // decoder_output = clip(frames, lo, hi) when clip_outputs (tacotron.py:360-361); the clip's
    // gradient passes where lo <= x <= hi (TF maximum/minimum)
    const float x = FR[i];
    const float y = clip ? fminf(fmaxf(x, lo), hi) : x;
    const float w = (!tlen || t < tlen[b]) ? 1.f : 0.f;
    const float d = (y - tg[((long)b * T + t) * NM + c]) * w;
    sq += d * d;
    const bool pass = !clip || (x >= lo && x <= hi);
    dFR[i] = pass ? 2.f * d * inv_f : 0.f;
    if (clipm) clipm[i] = pass ? 1 : 0;
    FR[i] = y;
  }
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < (long)T * B; i0 += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i0 % B), t = (int)(i0 / B);
    const long i = ((long)(t / r) * B + b) * r + t % r;
    const float x = ST[i], z = stg[(long)b * T + t];
    if (!tlen) {
      ce += fmaxf(x, 0.f) - x * z + log1pf(expf(-fabsf(x)));
      dST[i] = (sigm_acc(x) - z) * inv_s;
    } else {
      const float w = t < tlen[b] ? 1.f : 0.f;
      const float l = 1.f + (pos_weight - 1.f) * z;
      const float v = w * ((1.f - z) * x + l * (log1pf(expf(-fabsf(x))) + fmaxf(-x, 0.f)));
      ce += v;
      nz += v != 0.f ? 1.f : 0.f;
      dST[i] = w * ((1.f - z) - l * sigm_acc(-x));  // / count, by k_tr_div
    }
  }
  sq = block_sum(sq, s4);
  ce = block_sum(ce, s4);
  nz = block_sum(nz, s4);
  if (threadIdx.x == 0) {
    part[blockIdx.x * 3] = sq;
    part[blockIdx.x * 3 + 1] = ce;
    part[blockIdx.x * 3 + 2] = nz;
  }
}
// out[0] = before loss, out[1] = stop loss; masked (ns = 0): the stop normaliser is the count of
// nonzero masked losses, also stored in out[5] for k_tr_div
// fixed-order double tree over the 256 threads of the block (every thread calls it; result on all)
__device__ __forceinline__ double block_sum256_d(double v, double* sd) {
  const int tid = threadIdx.x;
  sd[tid] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) sd[tid] += sd[tid + o];
    __syncthreads();
  }
  const double r = sd[0];
  __syncthreads();
  return r;
}
__global__ __launch_bounds__(256) void k_tr_loss_final(const float* __restrict__ part, int nb, long nf, long ns,
                                                       float* __restrict__ out) {
  __shared__ double sd[256];
  double sq = 0, ce = 0, nz = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    sq += part[3 * i];
    ce += part[3 * i + 1];
    nz += part[3 * i + 2];
  }
  sq = block_sum256_d(sq, sd);
  ce = block_sum256_d(ce, sd);
  nz = block_sum256_d(nz, sd);
  if (threadIdx.x != 0) return;
  out[0] = (float)(sq / (double)nf);
  const double cnt = ns > 0 ? (double)ns : nz;
  out[1] = (float)(ce / cnt);
  out[5] = (float)cnt;
}
__global__ void k_tr_div(float* __restrict__ x, long n, const float* __restrict__ by) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] /= by[0];
}

// ---- backward ------------------------------------------------------------------------------
struct TrLstmBwd {
  const float* dh_ext;  // strided d h_new from the layer's consumers (or residual with part)
  long ld_dh;
  // non-null: d h_new = sum_z part[z][b][n] (+ dh_ext[b][n] if dh_ext) from a raw split-K GEMM
  // with pN columns; side != null also combines columns [H, 2H) (+ side_res) into side[b][n]
  const float* part;
  int ks;
  long pN;
  float* side;
  long ld_side;
  const float* side_res;
  long ld_side_res;
  const float* dhz;     // strided d(zoned h_t) from step t+1
  long ld_dhz;
  float* DC;            // [B,H] in: d(zoned c_t); out: d(zoned c_{t-1})
  const float* G;       // [B,4H] activations
  const float* cn;      // [B,H]
  const float* c_prev;  // [B,H]
  const uint8_t* zm;
  int t, layer, B, H;
  float z;
  float* dG;            // [B,4H]
  float* R;             // [B, ldr]: (1-kh)·dhz at column off_r + n
  long ldr;
  int off_r;
};
__global__ void k_tr_lstm_bwd(TrLstmBwd a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.B * a.H) return;
  const int b = i / a.H, n = i % a.H;
  const float* g = a.G + (long)b * 4 * a.H;
  const float si = g[n], tj = g[a.H + n], sf = g[2 * a.H + n], so = g[3 * a.H + n];
  float kc, kh;
  if (a.zm) {
    const long base = (((long)a.t * 4 + 2 * a.layer) * a.B + b) * a.H + n;
    kc = (float)a.zm[base];
    kh = (float)a.zm[base + (long)a.B * a.H];
  } else {
    kc = kh = 1.f - a.z;
  }
  const float dhz = a.dhz[(long)b * a.ld_dhz + n];
  const float dcz = a.DC[i];
  float dext;
  if (a.part) {
    dext = a.dh_ext ? a.dh_ext[(long)b * a.ld_dh + n] : 0.f;
    float sd = a.side ? a.side_res[(long)b * a.ld_side_res + a.H + n] : 0.f;
    const long zs = (long)a.B * a.pN;
    const float* p0 = a.part + (long)b * a.pN + n;
    if (a.side) {
#pragma unroll 4
      for (int z = 0; z < a.ks; ++z) {
        dext += p0[z * zs];
        sd += p0[z * zs + a.H];
      }
    } else {
#pragma unroll 4
      for (int z = 0; z < a.ks; ++z) dext += p0[z * zs];
    }
    if (a.side) a.side[(long)b * a.ld_side + n] = sd;
  } else {
    dext = a.dh_ext[(long)b * a.ld_dh + n];
  }
  const float dhn = dext + kh * dhz;
  const float cnew = a.cn[i];
  const float tc = tanhf(cnew);
  const float dcn = kc * dcz + dhn * so * (1.f - tc * tc);
  const float dso = dhn * tc, dsf = dcn * a.c_prev[i], dsi = dcn * tj, dtj = dcn * si;
  float* dg = a.dG + (long)b * 4 * a.H;
  dg[n] = dsi * si * (1.f - si);
  dg[a.H + n] = dtj * (1.f - tj * tj);
  dg[2 * a.H + n] = dsf * sf * (1.f - sf);
  dg[3 * a.H + n] = dso * so * (1.f - so);
  a.DC[i] = (1.f - kc) * dcz + dcn * sf;
  a.R[(long)b * a.ldr + a.off_r + n] = (1.f - kh) * dhz;
}

// ---- attention backward for one step: two chip-wide launches over (j-tile, row) ----
// (1) d align_j = dctx_t · values_j + d cum_t[j] (cum_t = cum_{t-1} + align_t), softmax backward
// de_j = a_j (da_j - Σ a·da), tanh backward du_jk = de_j v_k (1 - th²):
// d keys (+=), per-tile partials of d v_a, d b_a (= d q), du kept for d W_loc, d f = du · W_loc^T
__global__ __launch_bounds__(TR_AT) void k_tr_att_energy_bwd(TrAtt a) {
  __shared__ float WlT[256 * 33];
  __shared__ float dU[TR_JT * 256];
  __shared__ float de[TR_JT];
  __shared__ float racc[2 * TR_AT];
  __shared__ float s16[16];
  __shared__ __attribute__((aligned(16))) float dctx[1024];
  __shared__ float dat[TR_JT];
  const int b = blockIdx.y, tile = blockIdx.x, j0 = tile * TR_JT, tid = threadIdx.x;
  const long tb = (long)a.t * a.B + b;
  const int len = a.lens[b];
  // d context_t (block 0 keeps it for the d-values GEMM)
  for (int n = tid; n < a.D; n += blockDim.x) {
    const float v = a.dPIN[tb * (a.H + a.D) + a.H + n] + a.dX1[(tb + a.B) * (a.P + a.D + a.H) + a.P + n];
    dctx[n] = v;
    if (tile == 0) a.DCTX[tb * a.D + n] = v;
  }
  __syncthreads();
  // softmax backward needs s = Σ_j a_j da_j with da_j = dctx·v_j + dcum_j; since ctx_t = Σ_j a_j v_j,
  // s = dctx·ctx_t + Σ_j a_j dcum_j -- every tile gets it without the other tiles' da
  float s = 0.f;
  for (int n = tid; n < a.D; n += blockDim.x) s += dctx[n] * a.PIN[tb * (a.H + a.D) + a.H + n];
  for (int j = tid; j < len; j += blockDim.x) s += a.ALN[tb * a.Tin + j] * a.DCUM[(long)b * a.Tin + j];
  s = block_sum(s, s16);
  {  // d align of this tile's rows: one encoder row per wave
    const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    for (int jj = wave; jj < TR_JT; jj += nw) {
      const int j = j0 + jj;
      if (j >= a.Tin) break;
      const float* v = a.values + ((long)b * a.Tin + j) * a.D;
      float acc = 0.f;
      if ((a.D & 3) == 0) {  // 16-byte loads: the values row is the kernel's dominant read
        const float4* v4 = reinterpret_cast<const float4*>(v);
        const float4* d4 = reinterpret_cast<const float4*>(dctx);
#pragma unroll 4
        for (int n = lane; n < (a.D >> 2); n += 64) {
          const float4 x = v4[n], y = d4[n];
          acc += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
        }
      } else {
        for (int n = lane; n < a.D; n += 64) acc += dctx[n] * v[n];
      }
      acc = wave_sum(acc);
      if (lane == 0) dat[jj] = acc + a.DCUM[(long)b * a.Tin + j];
    }
  }
  __syncthreads();
  if (tid < TR_JT) {
    const int j = j0 + tid;
    const float aj = j < len ? a.ALN[tb * a.Tin + j] : 0.f;
    // smoothing: d e_j = a_j (d a_j - s)·(1 - sigmoid(e_j)), sigmoid(e_j) = a_j·Σ sigmoid
    de[tid] = j < len ? aj * (dat[tid] - s) * (a.smooth ? 1.f - aj * a.SS[tb] : 1.f) : 0.f;
  }
  for (int i = tid; i < a.F * a.A; i += blockDim.x) WlT[(i % a.A) * 33 + i / a.A] = a.Wl[i];
  __syncthreads();
  const int NJ = blockDim.x / a.A, k = tid % a.A, js = tid / a.A;
  const float vak = a.va[k];
  float dv = 0.f, dq = 0.f;
  for (int jj = js; jj < TR_JT; jj += NJ) {
    const int j = j0 + jj;
    float du = 0.f;
    if (j < a.Tin) {
      const long hidx = (tb * a.Tin + j) * a.A + k;
      const float th = a.TH[hidx];
      du = de[jj] * vak * (1.f - th * th);
      dv += de[jj] * th;
      dq += du;
      a.DKEYS[((long)b * a.Tin + j) * a.A + k] += du;
      a.TH[hidx] = du;  // d W_loc = FALL^T · du as one GEMM after the loop
    }
    dU[jj * a.A + k] = du;
  }
  racc[tid] = dv;
  racc[TR_AT + tid] = dq;
  __syncthreads();
  const long pt = (long)b * a.nt + tile;
  if (tid < a.A) {
    float sv = 0.f, sq = 0.f;
    for (int g = 0; g < NJ; ++g) {
      sv += racc[g * a.A + tid];
      sq += racc[TR_AT + g * a.A + tid];
    }
    a.PQ[pt * a.A + tid] = sq;
    a.dV[pt * a.A + tid] += sv;
    a.dBA[pt * a.A + tid] += sq;
  }
  for (int i = tid; i < TR_JT * a.F; i += blockDim.x) {
    const int jj = i / a.F, c = i % a.F, j = j0 + jj;
    if (j >= a.Tin) continue;
    float acc = 0.f;
    for (int kk = 0; kk < a.A; ++kk) acc += dU[jj * a.A + kk] * WlT[kk * 33 + c];
    a.DF[((long)b * a.Tin + j) * a.F + c] = acc;
  }
}

// Sum over all 64 lanes of each of 32 per-lane values (butterfly reduce-scatter, 32 shuffles): lane l
// returns the total of p[l >> 1].
__device__ __forceinline__ float wave_reduce_scatter32(float (&p)[32], int lane) {
  float q[16], r[8], u[4], v2[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool hi = lane & 32;
    q[i] = (hi ? p[16 + i] : p[i]) + __shfl_xor(hi ? p[i] : p[16 + i], 32, 64);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool hi = lane & 16;
    r[i] = (hi ? q[8 + i] : q[i]) + __shfl_xor(hi ? q[i] : q[8 + i], 16, 64);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool hi = lane & 8;
    u[i] = (hi ? r[4 + i] : r[i]) + __shfl_xor(hi ? r[i] : r[4 + i], 8, 64);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bool hi = lane & 4;
    v2[i] = (hi ? u[2 + i] : u[i]) + __shfl_xor(hi ? u[i] : u[2 + i], 4, 64);
  }
  const bool hi = lane & 2;
  const float x = (hi ? v2[1] : v2[0]) + __shfl_xor(hi ? v2[0] : v2[1], 2, 64);
  return x + __shfl_xor(x, 1, 64);
}

// k_tr_att_energy_bwd with 256 threads (A <= 128, F <= 32, D % 4 == 0, D <= 1024): wave w owns rows
// w + 4r of the tile; the lane's two W_loc columns in registers turn d f = du·W_locᵀ into 64 FMAs +
// one 32-value butterfly reduction per row instead of an LDS-staged transposed W_loc; every global
// operand of a row pair is loaded before its arithmetic.
__global__ __launch_bounds__(TR_E2T) void k_tr_att_energy_bwd2(TrAtt a) {
  __shared__ __attribute__((aligned(16))) float dctx[1024];
  __shared__ float racc[2][4][128];
  __shared__ float s16[16];
  const int b = blockIdx.y, tile = blockIdx.x, j0 = tile * TR_JT, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int F = a.F, A = a.A, Tin = a.Tin, D = a.D;
  const long tb = (long)a.t * a.B + b;
  const int len = a.lens[b];
  const int k0 = lane, k1 = lane + 64;
  const bool ok0 = k0 < A, ok1 = k1 < A;
  float wl0[32], wl1[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    wl0[c] = (c < F && ok0) ? a.Wl[c * A + k0] : 0.f;
    wl1[c] = (c < F && ok1) ? a.Wl[c * A + k1] : 0.f;
  }
  const float va0 = ok0 ? a.va[k0] : 0.f, va1 = ok1 ? a.va[k1] : 0.f;
  const long pt = (long)b * a.nt + tile;
  const float odv = tid < A ? a.dV[pt * A + tid] : 0.f, odb = tid < A ? a.dBA[pt * A + tid] : 0.f;
  float sp = 0.f;
  for (int n = tid; n < D; n += TR_E2T) {
    const float v = a.dPIN[tb * (a.H + D) + a.H + n] + a.dX1[(tb + a.B) * (a.P + D + a.H) + a.P + n];
    dctx[n] = v;
    if (tile == 0) a.DCTX[tb * D + n] = v;
    sp += v * a.PIN[tb * (a.H + D) + a.H + n];
  }
  // s = Σ_j a_j da_j = dctx·ctx_t + Σ_j a_j dcum_j (every tile gets it without the other tiles' da)
  for (int j = tid; j < len; j += TR_E2T) sp += a.ALN[tb * Tin + j] * a.DCUM[(long)b * Tin + j];
  const float s = block_sum(sp, s16);  // its barriers also publish dctx
  float dv0 = 0.f, dv1 = 0.f, dq0 = 0.f, dq1 = 0.f;
  const f32x4* d4 = reinterpret_cast<const f32x4*>(dctx);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = j0 + w + 4 * r;
    if (j >= Tin) break;
    // d align_j = dctx·values_j + d cum_t[j] (16-byte loads of the values row: the dominant read)
    const f32x4* v4 = reinterpret_cast<const f32x4*>(a.values + ((long)b * Tin + j) * D);
    f32x4 vv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) vv[i] = (lane + 64 * i) * 4 < D ? v4[lane + 64 * i] : f32x4{0.f, 0.f, 0.f, 0.f};
    const long hrow = (tb * Tin + j) * A, krow = ((long)b * Tin + j) * A;
    const float th0 = ok0 ? a.TH[hrow + k0] : 0.f, th1 = ok1 ? a.TH[hrow + k1] : 0.f;
    const float dk0 = ok0 ? a.DKEYS[krow + k0] : 0.f, dk1 = ok1 ? a.DKEYS[krow + k1] : 0.f;
    const float aln = a.ALN[tb * Tin + j], dcum = a.DCUM[(long)b * Tin + j];
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if ((lane + 64 * i) * 4 < D) {
        const f32x4 y = d4[lane + 64 * i];
        acc += vv[i][0] * y[0] + vv[i][1] * y[1] + vv[i][2] * y[2] + vv[i][3] * y[3];
      }
    }
    acc = wave_sum(acc);
    const float de = j < len ? aln * ((acc + dcum) - s) * (a.smooth ? 1.f - aln * a.SS[tb] : 1.f) : 0.f;
    const float du0 = de * va0 * (1.f - th0 * th0), du1 = de * va1 * (1.f - th1 * th1);
    dv0 += de * th0;
    dv1 += de * th1;
    dq0 += du0;
    dq1 += du1;
    if (ok0) {
      a.DKEYS[krow + k0] = dk0 + du0;
      a.TH[hrow + k0] = du0;  // d W_loc = FALL^T · du after the loop
    }
    if (ok1) {
      a.DKEYS[krow + k1] = dk1 + du1;
      a.TH[hrow + k1] = du1;
    }
    float p[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) p[c] = du0 * wl0[c] + du1 * wl1[c];
    const float dfc = wave_reduce_scatter32(p, lane);
    if ((lane & 1) == 0 && (lane >> 1) < F) a.DF[((long)b * Tin + j) * F + (lane >> 1)] = dfc;
  }
  if (ok0) {
    racc[0][w][k0] = dv0;
    racc[1][w][k0] = dq0;
  }
  if (ok1) {
    racc[0][w][k1] = dv1;
    racc[1][w][k1] = dq1;
  }
  __syncthreads();
  if (tid < A) {
    const float sv = (racc[0][0][tid] + racc[0][1][tid]) + (racc[0][2][tid] + racc[0][3][tid]);
    const float sq = (racc[1][0][tid] + racc[1][1][tid]) + (racc[1][2][tid] + racc[1][3][tid]);
    a.PQ[pt * A + tid] = sq;
    a.dV[pt * A + tid] = odv + sv;
    a.dBA[pt * A + tid] = odb + sq;
  }
}

// (2) d query (sum of the tile partials), location-conv backward: per-tile partials of d Kc and
// d bc, and d cum_{t-1}[i] = d cum_t[i] + Σ_tap,c df[i - tap + pad][c]·Kc[tap][c]
__global__ __launch_bounds__(256) void k_tr_att_conv_bwd(TrAtt a) {
  __shared__ float cseg[TR_JT + 64];
  __shared__ float dfh[(TR_JT + 64) * 32];
  __shared__ float Kcs[65 * 32];  // conv taps from LDS: the d cum loop runs KW dependent steps
  const int b = blockIdx.y, tile = blockIdx.x, j0 = tile * TR_JT, tid = threadIdx.x;
  const int pad = (a.KW - 1) / 2, lo = a.KW - 1 - pad;  // halo below / above
  const long tb = (long)a.t * a.B + b;
  const long pt = (long)b * a.nt + tile;
  // the accumulators' old values are loaded with the staging loads: one memory round trip before
  // the arithmetic instead of one per read-modify-write (KW·F <= 65·32 = 8 per thread)
  constexpr int KCM = (65 * 32 + 255) / 256;
  float okc[KCM];
#pragma unroll
  for (int u = 0; u < KCM; ++u) {
    const int i = tid + 256 * u;
    okc[u] = i < a.KW * a.F ? a.dKC[pt * a.KW * a.F + i] : 0.f;
  }
  const float obc = tid < a.F ? a.dBC[pt * a.F + tid] : 0.f;
  float dq = 0.f;
  if (tile == 0 && tid < a.A)
    for (int g = 0; g < a.nt; ++g) dq += a.PQ[((long)b * a.nt + g) * a.A + tid];
  const float* cum_prev = a.CUM + tb * a.Tin;
  for (int i = tid; i < TR_JT + a.KW - 1; i += blockDim.x) {
    const int j = j0 + i - pad;
    cseg[i] = (j >= 0 && j < a.Tin) ? cum_prev[j] : 0.f;
  }
  // df rows j0 - lo .. j0 + TR_JT - 1 + pad (zero outside [0, Tin))
  const int nh = TR_JT + a.KW - 1;
  for (int i = tid; i < nh * a.F; i += blockDim.x) {
    const int j = j0 - lo + i / a.F, c = i % a.F;
    dfh[i] = (j >= 0 && j < a.Tin) ? a.DF[((long)b * a.Tin + j) * a.F + c] : 0.f;
  }
  // 32 lanes per position (lane = filter), 8 positions per pass: old d cum values first
  const int c32 = tid & 31;
  float odc[TR_JT / 8];
#pragma unroll
  for (int u = 0; u < TR_JT / 8; ++u) {
    const int i = j0 + 8 * u + tid / 32;
    odc[u] = (c32 == 0 && i < a.Tin) ? a.DCUM[(long)b * a.Tin + i] : 0.f;
  }
  for (int i = tid; i < a.KW * a.F; i += blockDim.x) Kcs[i] = a.Kc[i];
  if (tile == 0 && tid < a.A) a.DQ[tb * a.A + tid] = dq;
  __syncthreads();
  const float* dfs = dfh + lo * a.F;  // the tile's own rows
#pragma unroll
  for (int u = 0; u < KCM; ++u) {
    const int i = tid + 256 * u;
    if (i < a.KW * a.F) {
      const int tap = i / a.F, c = i % a.F;
      float acc = 0.f;
      for (int jj = 0; jj < TR_JT; ++jj) acc += dfs[jj * a.F + c] * cseg[jj + tap];
      a.dKC[pt * a.KW * a.F + i] = okc[u] + acc;
    }
  }
  if (tid < a.F) {
    float acc = 0.f;
    for (int jj = 0; jj < TR_JT; ++jj) acc += dfs[jj * a.F + tid];
    a.dBC[pt * a.F + tid] = obc + acc;
  }
#pragma unroll
  for (int u = 0; u < TR_JT / 8; ++u) {
    const int ii = 8 * u + tid / 32, i = j0 + ii;
    float acc = 0.f;
    if (c32 < a.F)
      for (int tap = 0; tap < a.KW; ++tap) acc += dfs[(ii - tap + pad) * a.F + c32] * Kcs[tap * a.F + c32];
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (c32 == 0 && i < a.Tin) a.DCUM[(long)b * a.Tin + i] = odc[u] + acc;
  }
}

// The whole attention backward of one step (k_tr_att_energy_bwd2 + k_tr_att_conv_bwd) in ONE launch of
// nq <= 4 work-groups per row (256 work-groups at B = 64): work-group (q, b) owns the positions
// [j0, j1) of row b.  The location-conv backward into d cum crosses positions; it is deferred by one
// step so no work-group waits for another in the same launch:
//   d cum_t[i] = d cum_{t+1}[i] + Σ_tap,c df_{t+1}[i - tap + pad][c]·Kc[tap][c]
// is formed for the own positions from the previous launch's df (the rows [j0 - pad, j1 + pad)), and
// the full-row Σ_i a_t[i]·d cum_t[i] of the softmax backward as Σ_i a_t[i]·d cum_{t+1}[i] plus the
// previous launch's per-range partials Σ_{j'} Σ_c df_{t+1}[j'][c]·Σ_tap a_t[j' + tap - pad]·Kc[tap][c]
// (the same sum with the conv moved onto the alignments).  d cum, df, those partials and the d query
// partials are double-buffered by step parity; the LSTM-2 backward of the step sums the nq d query
// partials of its A-operand rows itself (TrFused::af_parts) and the next launch writes the step's sum
// to DQ (for the query-layer kernel gradient after the loop).
//   d align_j = dctx·values_j + d cum_j (the bf16 values copy the forward's context read, when present)
//   de_j = a_j (d align_j - s), du_jk = de_j v_k (1 - th_jk²), d keys += du, d v_a, d b_a
//   df = du·W_locᵀ and the d Kc partial Σ_j df[j][c]·cum_{t-1}[j + tap - pad] on fp32 MFMA
//   (v_mfma_f32_16x16x4f32: exact fp32 products); cross-lane sums by DPP (no LDS round trips)
constexpr int TRQ_NT = 256;
constexpr int TRQ_RB = 16;  // own rows per wave per batch of loads
typedef float trq_f4 __attribute__((ext_vector_type(4)));
struct TrQ {
  int nq;
  const float* dcum_in;  // [B][Tin] d cum input of the previous launch (full rows)
  const float* df_in;    // [B][Tin][F] df of the previous launch
  const float* pq_in;    // [B][nt][A] d query partials of the previous launch
  const float* sc_in;    // [B][4] the previous launch's conv-moved Σ a·d cum partials
  float *dcum_out, *df_out, *pq_out, *sc_out;
};
template <int CTRL, int RMASK>
__device__ __forceinline__ float trq_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, RMASK, 0xf, false));
}
// sum of the 16 lanes of each row, in every lane of the row (xor 1, xor 2, half mirror, mirror)
__device__ __forceinline__ float trq_row_sum(float v) {
  v += trq_dpp<0xB1, 0xf>(v);
  v += trq_dpp<0x4E, 0xf>(v);
  v += trq_dpp<0x141, 0xf>(v);
  v += trq_dpp<0x140, 0xf>(v);
  return v;
}
// wave sum (uniform result): row sums, rows chained by row_bcast:15 / row_bcast:31 into lane 63
__device__ __forceinline__ float trq_wave_sum(float v) {
  v = trq_row_sum(v);
  v += trq_dpp<0x142, 0xa>(v);
  v += trq_dpp<0x143, 0xc>(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__global__ __launch_bounds__(TRQ_NT, 1) void k_tr_att_bwd_q(TrAtt a, TrQ z) {
  constexpr int A = 128, F = 32, KW = 31, PAD = 15, NW = TRQ_NT / 64, TMX = 256, RQX = 64, HR = RQX + 2 * PAD + 2;
  __shared__ __attribute__((aligned(16))) float dctx[1024];
  constexpr int WLS = A + 4;                                  // padded W_loc rows: conflict-free A fragments
  __shared__ __attribute__((aligned(16))) float wls[F * WLS];  // W_loc [c][k]
  __shared__ __attribute__((aligned(16))) float kcs[32 * F];  // Kc [tap][c] (tap 31 zero)
  __shared__ __attribute__((aligned(16))) float dfin[HR * F]; // previous df, row r = position j0 - pad - 1 + r
  __shared__ float alns[TMX];                                 // a_t
  __shared__ float dcin[TMX];                                 // d cum_{t+1}
  __shared__ float alnh[RQX + 32];                            // a_{t-1}[j0 - pad + i] (the next step's alignments)
  __shared__ float dcum[RQX];                                 // d cum_t of the own rows
  __shared__ float de[RQX];
  __shared__ float dus[RQX * (A + 1)];                        // du of the own rows (stride A + 1)
  __shared__ float dfo[RQX * F];                              // this launch's df of the own rows (zero past nown)
  __shared__ float cseg[RQX + 32];                            // cum_{t-1}[j0 + i - pad]
  constexpr int MSS = 33;                                     // stride of ms: conflict-free diagonal reads
  __shared__ float ms[HR * MSS];                              // M[r][tap] = Σ_c df_{t+1}[r][c]·Kc[tap][c]
  __shared__ float red[2][NW][A];
  __shared__ float s16[16];
  const int q = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Tin = a.Tin, D = a.D, nq = z.nq;
  const long tb = (long)a.t * a.B + b;
  const int len = a.lens[b];
  const int RQ = (Tin + nq - 1) / nq, j0 = min(Tin, q * RQ), j1 = min(Tin, j0 + RQ), nown = j1 - j0;
  const int k0 = lane, k1 = lane + 64;
  const int jl = lane & 15, g4 = lane >> 4;
  long long* const stp = (a.stamps && a.t == a.stamp_t && tid == 0) ? a.stamps + ((long)b * 4 + q) * 16 : nullptr;
#define TRQ_STAMP(i) \
  if (stp) stp[i] = __builtin_amdgcn_s_memrealtime()
  TRQ_STAMP(0);
  const long pt = (long)b * a.nt + q;
  // ---- staging: every load of the prologue in flight at once (16-byte loads where the rows allow)
  const trq_f4 zf4 = {0.f, 0.f, 0.f, 0.f};
  // every load below is unconditional (clamped address, the value selected afterwards): a load under a
  // branch makes the wait-count pass fall back to vmcnt(0) at the join, serialising the round trips
  const bool d4ok = tid * 4 < D;  // host: D % 4 == 0, D <= 1024
  const int n4 = d4ok ? 4 * tid : 0;
  const long ofs_p = tb * (a.H + D) + a.H, ofs_x = (tb + a.B) * (a.P + D + a.H) + a.P;
  trq_f4 xp = *reinterpret_cast<const trq_f4*>(a.dPIN + ofs_p + n4);
  trq_f4 xx = *reinterpret_cast<const trq_f4*>(a.dX1 + ofs_x + n4);
  trq_f4 xc = *reinterpret_cast<const trq_f4*>(a.PIN + ofs_p + n4);
  trq_f4 wlv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) wlv[u] = reinterpret_cast<const trq_f4*>(a.Wl)[tid + TRQ_NT * u];
  trq_f4 kcv = reinterpret_cast<const trq_f4*>(a.Kc)[min(tid, KW * F / 4 - 1)];
  constexpr int NH = (HR * F / 4 + TRQ_NT - 1) / TRQ_NT;
  trq_f4 dfv[NH];
  bool dfok[NH];
  const float* dfrow = z.df_in + (long)b * Tin * F;
#pragma unroll
  for (int u = 0; u < NH; ++u) {
    const int i4 = tid + TRQ_NT * u, r = i4 / (F / 4), j = j0 - PAD - 1 + r;
    dfok[u] = i4 < HR * F / 4 && j >= 0 && j < Tin;
    dfv[u] = reinterpret_cast<const trq_f4*>(dfrow + (long)(dfok[u] ? j : 0) * F)[i4 % (F / 4)];
  }
  const int tc = min(tid, Tin - 1);
  float aln_v = a.ALN[tb * Tin + tc];
  float dci_v = z.dcum_in[(long)b * Tin + tc];
  const int jc = j0 + tid - PAD;
  const bool hal = tid < RQX + 32 && jc >= 0 && jc < Tin;
  const int jcc = hal ? jc : 0;
  float cs_v = a.CUM[tb * Tin + jcc];
  float an_v = a.ALN[(a.t > 0 ? tb - a.B : tb) * Tin + jcc];
  float scp[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) scp[g] = z.sc_in[(long)b * 4 + min(g, nq - 1)];
  const int ta = min(tid, A - 1), tf = min(tid, F - 1);
  float odv = a.dV[pt * A + ta], odb = a.dBA[pt * A + ta];
  float obc = a.dBC[pt * F + tf];
  // the d Kc slot entries of this lane's MFMA output (wave w < 4: tap tile w >> 1, filter tile w & 1)
  const int kt0 = 16 * (w >> 1) + 4 * g4, kcc = 16 * (w & 1) + jl;
  float okc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) okc[i] = a.dKC[pt * KW * F + min(kt0 + i, KW - 1) * F + kcc];
  // the d W_loc accumulator entries of this lane: wave w owns the G tiles w + 4u (tap tile tl >> 3,
  // column tile tl & 7), MFMA D rows 4 g4 + i, column jl
  float* const dwg = a.DWGP + pt * 32 * A;
  float odw[16];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int tl = w + 4 * u;
      odw[4 * u + i] = dwg[(16 * (tl >> 3) + 4 * g4 + i) * A + 16 * (tl & 7) + jl];
    }
  // d query of step t + 1 = the sum of that launch's partials (in range order), written by q == 0
  const bool dq_prev = q == 0 && tid < A && a.t + 1 < a.T;
  float pqv[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) pqv[g] = z.pq_in[((long)b * a.nt + min(g, nq - 1)) * A + ta];
  // ---- the own rows' values (bf16 step) and tanh / d keys rows, behind the staging loads: their round
  // trip overlaps the d cum phase (wave w: rows jr = w + NW u, clamped to the last own row)
  typedef unsigned trq_u4 __attribute__((ext_vector_type(4)));
  const bool v16 = a.values16 && (a.D & 7) == 0;
  trq_u4 vv[TRQ_RB][2];
  float t0[TRQ_RB], t1[TRQ_RB], e0[TRQ_RB], e1[TRQ_RB];
  if (nown > 0) {
    const __bf16* vbase = v16 ? a.values16 : reinterpret_cast<const __bf16*>(a.values);  // any valid row
#pragma unroll
    for (int u = 0; u < TRQ_RB; ++u) {
      const int jr = min(w + NW * u, nown - 1);
      const trq_u4* v8 = reinterpret_cast<const trq_u4*>(vbase + ((long)b * Tin + j0 + jr) * D);
#pragma unroll
      for (int i = 0; i < 2; ++i) vv[u][i] = v8[min(lane + 64 * i, D / 8 - 1)];
      const long hrow = (tb * Tin + j0 + jr) * A, krow = ((long)b * Tin + j0 + jr) * A;
      t0[u] = a.TH[hrow + k0];
      t1[u] = a.TH[hrow + k1];
      e0[u] = a.DKEYS[krow + k0];
      e1[u] = a.DKEYS[krow + k1];
    }
  }
  // the selections of the clamped loads
  if (!d4ok) xp = xx = xc = zf4;
  if (tid >= KW * F / 4) kcv = zf4;
#pragma unroll
  for (int u = 0; u < NH; ++u)
    if (!dfok[u]) dfv[u] = zf4;
  if (tid >= Tin) aln_v = dci_v = 0.f;
  if (!hal) cs_v = 0.f;
  if (!hal || a.t == 0) an_v = 0.f;
  float scv = 0.f;
#pragma unroll
  for (int g = 0; g < 4; ++g) scv += g < nq ? scp[g] : 0.f;
  // ---- LDS writes
  float sp = 0.f;
  if (d4ok) {
    const trq_f4 v = xp + xx;
    *reinterpret_cast<trq_f4*>(dctx + 4 * tid) = v;
    sp = v[0] * xc[0] + v[1] * xc[1] + v[2] * xc[2] + v[3] * xc[3];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i4 = tid + TRQ_NT * u;  // W_loc element 4 i4 = row i4 / 32, column 4 (i4 % 32)
    *reinterpret_cast<trq_f4*>(wls + (i4 >> 5) * WLS + 4 * (i4 & 31)) = wlv[u];
  }
  reinterpret_cast<trq_f4*>(kcs)[tid] = kcv;  // 256 x 4 = 32 x F: the tap-31 row zero
#pragma unroll
  for (int u = 0; u < NH; ++u) {
    const int i4 = tid + TRQ_NT * u;
    if (i4 < HR * F / 4) reinterpret_cast<trq_f4*>(dfin)[i4] = dfv[u];
  }
  alns[tid] = aln_v;
  dcin[tid] = dci_v;
  if (tid < RQX + 32) {
    cseg[tid] = cs_v;
    alnh[tid] = an_v;
  }
  for (int i = tid; i < RQX * F; i += TRQ_NT) dfo[i] = 0.f;
  sp += aln_v * dci_v;  // Σ_i a_t[i] d cum_{t+1}[i] (a_t = 0 past the length)
  __syncthreads();
  TRQ_STAMP(1);
  // ---- d cum_t of the own rows: 32 lanes (filters c, taps in registers) per position, then across the
  // filters by DPP (lanes 31 / 63 hold positions p, p + 1)
  float kcr[KW];
#pragma unroll
  for (int tp = 0; tp < KW; ++tp) kcr[tp] = kcs[tp * F + (tid & 31)];
  // d cum_t[ir] = d cum_{t+1}[ir] + Σ_tap M[ir - tap + 2 pad + 1][tap]: M = dfin·Kcᵀ on fp32 MFMA
  // (v_mfma_f32_16x16x4f32, tile = 16 halo rows x 16 taps, K = the 32 filters), then the diagonal sums
  // from LDS, a quad of lanes per own row (8 taps each)
  {
    const int nrt = min(HR / 16, (nown + 2 * PAD + 1 + 15) / 16);
    for (int tl = w; tl < 2 * nrt; tl += NW) {
      const int rt = tl >> 1, tt = tl & 1;
      trq_f4 acc = {};
#pragma unroll
      for (int ks = 0; ks < F / 4; ++ks)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dfin[(16 * rt + jl) * F + 4 * ks + g4], kcs[(16 * tt + jl) * F + 4 * ks + g4],
                                                   acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) ms[(16 * rt + 4 * g4 + i) * MSS + 16 * tt + jl] = acc[i];
    }
  }
  __syncthreads();
  for (int p0 = 0; p0 < nown; p0 += TRQ_NT / 4) {
    const int ir = p0 + (tid >> 2), qq = tid & 3;  // own row, taps [8 qq, 8 qq + 8)
    float acc = 0.f;
    if (ir < nown) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int tp = 8 * qq + k;
        if (tp < KW) acc += ms[(ir - tp + 2 * PAD + 1) * MSS + tp];
      }
    }
    acc += trq_dpp<0xB1, 0xf>(acc);
    acc += trq_dpp<0x4E, 0xf>(acc);
    if (qq == 0 && ir < nown) {
      const float v = dcin[j0 + ir] + acc;
      dcum[ir] = v;
      z.dcum_out[(long)b * Tin + j0 + ir] = v;
    }
  }
  TRQ_STAMP(2);
  // s = Σ_j a_j da_j = dctx·ctx_t + Σ_j a_j d cum_t[j]   (block_sum's barriers also publish dcum)
  const float s = block_sum(sp, s16) + scv;
  const float ssum = a.smooth ? a.SS[tb] : 0.f;  // smoothing: Σ sigmoid(e) of this step
  TRQ_STAMP(3);
  // ---- d align of the own rows (jr = w + NW u): every row's values in flight before the dot products
  const trq_f4* d4 = reinterpret_cast<const trq_f4*>(dctx);
  if (v16) {
    trq_f4 dc[4];  // channels 8 (lane + 64 i) .. +8
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool ok = (lane + 64 * i) * 8 < D;
      dc[2 * i] = ok ? d4[2 * (lane + 64 * i)] : zf4;
      dc[2 * i + 1] = ok ? d4[2 * (lane + 64 * i) + 1] : zf4;
    }
#pragma unroll
    for (int u = 0; u < TRQ_RB; ++u) {
      const int jr = w + NW * u;
      if (jr >= nown) break;  // wave-uniform
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const unsigned x0 = vv[u][i][2 * h], x1 = vv[u][i][2 * h + 1];
          const trq_f4 y = dc[2 * i + h];  // zero for channel chunks past D (the clamped loads' duplicates)
          acc += __uint_as_float(x0 << 16) * y[0] + __uint_as_float(x0 & 0xffff0000u) * y[1] +
                 __uint_as_float(x1 << 16) * y[2] + __uint_as_float(x1 & 0xffff0000u) * y[3];
        }
      acc = trq_wave_sum(acc);
      if (lane == 0) {
        const int j = j0 + jr;
        de[jr] = j < len ? alns[j] * ((acc + dcum[jr]) - s) * (a.smooth ? 1.f - alns[j] * ssum : 1.f) : 0.f;
      }
    }
  } else {
    trq_f4 dc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dc[i] = (lane + 64 * i) * 4 < D ? d4[lane + 64 * i] : zf4;
    for (int r0 = w; r0 < nown; r0 += NW * (TRQ_RB / 2)) {
      trq_f4 vv[TRQ_RB / 2][4];
#pragma unroll
      for (int u = 0; u < TRQ_RB / 2; ++u) {
        const int jr = r0 + NW * u;
        const bool ok = jr < nown;
        const trq_f4* v4 = reinterpret_cast<const trq_f4*>(a.values + ((long)b * Tin + j0 + (ok ? jr : 0)) * D);
#pragma unroll
        for (int i = 0; i < 4; ++i) vv[u][i] = (ok && (lane + 64 * i) * 4 < D) ? v4[lane + 64 * i] : zf4;
      }
#pragma unroll
      for (int u = 0; u < TRQ_RB / 2; ++u) {
        const int jr = r0 + NW * u;
        if (jr >= nown) break;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc += vv[u][i][0] * dc[i][0] + vv[u][i][1] * dc[i][1] + vv[u][i][2] * dc[i][2] + vv[u][i][3] * dc[i][3];
        acc = trq_wave_sum(acc);
        if (lane == 0) {
          const int j = j0 + jr;
          de[jr] = j < len ? alns[j] * ((acc + dcum[jr]) - s) * (a.smooth ? 1.f - alns[j] * ssum : 1.f) : 0.f;
        }
      }
    }
  }
  __syncthreads();
  TRQ_STAMP(4);
  // ---- tanh backward, d keys, d v_a / d b_a partials of the own rows; du -> LDS
  const float va0 = a.va[k0], va1 = a.va[k1];
  float dv0 = 0.f, dv1 = 0.f, dq0 = 0.f, dq1 = 0.f;
#pragma unroll
  for (int u = 0; u < TRQ_RB; ++u) {
    const int jr = w + NW * u;
    if (jr >= nown) break;  // wave-uniform
    const long hrow = (tb * Tin + j0 + jr) * A, krow = ((long)b * Tin + j0 + jr) * A;
    const float dej = de[jr];
    const float du0 = dej * va0 * (1.f - t0[u] * t0[u]), du1 = dej * va1 * (1.f - t1[u] * t1[u]);
    dv0 += dej * t0[u];
    dv1 += dej * t1[u];
    dq0 += du0;
    dq1 += du1;
    a.DKEYS[krow + k0] = e0[u] + du0;
    a.DKEYS[krow + k1] = e1[u] + du1;
    dus[jr * (A + 1) + k0] = du0;
    dus[jr * (A + 1) + k1] = du1;
  }
  for (int i = nown * (A + 1) + tid; i < RQX * (A + 1); i += TRQ_NT) dus[i] = 0.f;
  red[0][w][k0] = dv0;
  red[0][w][k1] = dv1;
  red[1][w][k0] = dq0;
  red[1][w][k1] = dq1;
  __syncthreads();
  TRQ_STAMP(5);
  if (tid < A) {
    const float sv = (red[0][0][tid] + red[0][1][tid]) + (red[0][2][tid] + red[0][3][tid]);
    const float sq = (red[1][0][tid] + red[1][1][tid]) + (red[1][2][tid] + red[1][3][tid]);
    a.dV[pt * A + tid] = odv + sv;
    a.dBA[pt * A + tid] = odb + sq;
    z.pq_out[pt * A + tid] = sq;
  }
  // ---- d W_loc through the cumulative alignments, accumulated over the steps in this work-group's
  // slot (no du stream to HBM, no pass after the loop): G[tap][a] += Σ_jr cseg[jr + tap]·du[jr][a] on
  // fp32 MFMA; A [tap = 16 mt + jl][jr = 4 ks + g4] from cseg, B [jr][a = 16 nt + jl] from dus (zero past
  // nown).  Row 31 (no tap) is Σ du = d b_a, filled after the loop.
  {
    const int nk = (nown + 3) >> 2;
    trq_f4 gacc[4] = {};
    for (int ks = 0; ks < nk; ++ks) {
      const int jr = 4 * ks + g4;
      const float* dr = dus + jr * (A + 1) + jl;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int tl = w + 4 * u;
        gacc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(cseg[jr + 16 * (tl >> 3) + jl], dr[16 * (tl & 7)], gacc[u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tl = w + 4 * u;
        dwg[(16 * (tl >> 3) + 4 * g4 + i) * A + 16 * (tl & 7) + jl] = odw[4 * u + i] + gacc[u][i];
      }
  }
  // ---- df^T[c][j] = Σ_k W_loc[c][k] du[j][k]: wave w owns the position tile 16 w (16 rows), both
  // filter tiles; A [c = 16 mt + jl][k = 4 ks + g4] from wls, B [k][j = 16 w + jl] from dus
  if (16 * w < nown) {
    trq_f4 acc[2] = {};
    const float* dr = dus + (16 * w + jl) * (A + 1) + g4;
#pragma unroll
    for (int ks = 0; ks < 32; ++ks) {
      const float bv = dr[4 * ks];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wls[(16 * mt + jl) * WLS + 4 * ks + g4], bv, acc[mt], 0, 0, 0);
    }
    const int jr = 16 * w + jl;
    if (jr < nown) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int c0 = 16 * mt + 4 * g4;
        *reinterpret_cast<trq_f4*>(dfo + jr * F + c0) = acc[mt];
        *reinterpret_cast<trq_f4*>(z.df_out + ((long)b * Tin + j0 + jr) * F + c0) = acc[mt];
      }
    }
  }
  __syncthreads();
  TRQ_STAMP(6);
  // ---- d Kc partial [tap][c] = Σ_jr cseg[jr + tap]·dfo[jr][c]: wave w -> tap tile w >> 1, filter
  // tile w & 1; A [tap = 16 mt + jl][jr = 4 ks + g4], B [jr = 4 ks + g4][c = 16 nt + jl]
  {
    const int mt = w >> 1, nt = w & 1;
    trq_f4 acc = {};
#pragma unroll
    for (int ks = 0; ks < RQX / 4; ++ks) {
      const int jr = 4 * ks + g4;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(cseg[jr + 16 * mt + jl], dfo[jr * F + 16 * nt + jl], acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (kt0 + i < KW) a.dKC[pt * KW * F + (kt0 + i) * F + kcc] = okc[i] + acc[i];
  }
  // ---- d bc partial and the next launch's conv-moved partial Σ_jr Σ_c df[jr][c]·Σ_tap a_{t-1}[j0 + jr +
  // tap - pad]·Kc[tap][c]: thread (c = tid & 31, row group tid >> 5)
  {
    const int c = tid & 31, gq = tid >> 5;
    float accb = 0.f, accs = 0.f;
    for (int jr = gq; jr < nown; jr += 8) {
      const float dfv1 = dfo[jr * F + c];
      accb += dfv1;
      float g = 0.f;
#pragma unroll
      for (int tp = 0; tp < KW; ++tp) g += alnh[jr + tp] * kcr[tp];
      accs += dfv1 * g;
    }
    float* const rbc = &red[0][0][0];  // free again: read before the df barrier
    rbc[tid] = accb;
    rbc[TRQ_NT + tid] = accs;
    __syncthreads();
    if (tid < F) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) v += rbc[g * 32 + tid];
      a.dBC[pt * F + tid] = obc + v;
    }
    if (w == 1) {  // one wave: Σ over the 256 partials
      float v = rbc[TRQ_NT + lane] + rbc[TRQ_NT + 64 + lane] + rbc[TRQ_NT + 128 + lane] + rbc[TRQ_NT + 192 + lane];
      v = trq_wave_sum(v);
      if (lane == 0) z.sc_out[(long)b * 4 + q] = v;
    }
  }
  if (q == 0)  // stored last: a store ahead of the loads would hold up their waits (one vmcnt counter)
    for (int n = tid; n < D; n += TRQ_NT) a.DCTX[tb * D + n] = dctx[n];
  if (dq_prev) {
    float dq = 0.f;
    for (int g = 0; g < nq; ++g) dq += pqv[g];
    a.DQ[(tb + a.B) * A + tid] = dq;
  }
  TRQ_STAMP(7);
#undef TRQ_STAMP
}

// d query of the last backward launch (step 0): the sum of its position-range partials
__global__ void k_tr_dq_sum(const float* __restrict__ pq, int nt, int nq, int A, float* __restrict__ dq) {
  const int b = blockIdx.x;
  for (int k = threadIdx.x; k < A; k += blockDim.x) {
    float v = 0.f;
    for (int g = 0; g < nq; ++g) v += pq[((long)b * nt + g) * A + k];
    dq[(long)b * A + k] = v;
  }
}

// d W_loc (location_features_layer, attention.py:59-62) = Σ_r f[r][c]·du[r][k] over all R = T·B·T_in
// rows of FALL [R][F] and the du copy in TH [R][A], on fp32 MFMA (v_mfma_f32_32x32x2f32, exact fp32
// products): one streaming pass over the two fp32 arrays instead of a transpose, two bf16 copies and a
// K = R library GEMM.  Work-group = 4 waves, wave w owns output columns [32w, 32w+32) (A <= 128,
// F <= 32); rows [blockIdx.x·rpb, +rpb), 16 row pairs per round with every load issued first;
// partial [F][A] per work-group (summed by tr_colsum).
typedef float tr_f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(256) void k_tr_dwloc(const float* __restrict__ f, const float* __restrict__ du, long R,
                                                  int F, int A, long rpb, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  const int c = lane & 31, h = lane >> 5, k = 32 * w + (lane & 31);
  const bool cok = c < F, kok = k < A;
  tr_f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  for (long rb = r0; rb < r1; rb += 32) {
    float av[16], bv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const long rr = rb + 2 * u + h;
      const bool ok = rr < r1;
      av[u] = (ok && cok) ? f[rr * F + c] : 0.f;
      bv[u] = (ok && kok) ? du[rr * A + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
  // D: column k (lane & 31), row c' = (q & 3) + 8 (q >> 2) + 4h
  float* P = part + (long)blockIdx.x * F * A;
  if (kok)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int cr = (q & 3) + 8 * (q >> 2) + 4 * h;
      if (cr < F) P[(long)cr * A + k] = acc[q];
    }
}

// d W_loc without the location features: f = bc + conv(cum_{t-1}, Kc) is linear in Kc and bc, so
//   d W_loc[c][a] = bc[c]·Σ_r du[r][a] + Σ_tap Kc[tap][c]·G[tap][a],  G[tap][a] = Σ_r cum_{t-1}[j + tap - pad]·du[r][a]
// over all rows r = (t, b, j).  k_tr_dwloc's streaming fp32-MFMA pass with the A operand generated from
// the cumulative alignments (rows tap < KW; row 31 = 1, the Σ du row): one read of du and no FALL
// (T·B·T_in·F floats written by the forward, read back here).
__global__ __launch_bounds__(256) void k_tr_dwloc_cum(const float* __restrict__ CUM, const float* __restrict__ du,
                                                      long R, int Tin, int A, int KW, long rpb, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  const int c = lane & 31, h = lane >> 5, k = 32 * w + (lane & 31);
  const bool kok = k < A;
  const int pad = (KW - 1) / 2;
  tr_f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  int jb = (int)(r0 % Tin);  // position of row rb (one 64-bit remainder per work-group)
  for (long rb = r0; rb < r1; rb += 32) {
    float av[16], bv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const long rr = rb + 2 * u + h;
      const bool ok = rr < r1;
      int j = jb + 2 * u + h;
      while (j >= Tin) j -= Tin;
      const int jj = j + c - pad;
      const bool cv = ok && c < KW && jj >= 0 && jj < Tin;
      const float x = CUM[cv ? rr - j + jj : 0];
      av[u] = cv ? x : (ok && c == 31 ? 1.f : 0.f);
      bv[u] = (ok && kok) ? du[rr * A + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
    jb += 32;
    while (jb >= Tin) jb -= Tin;
  }
  float* P = part + (long)blockIdx.x * 32 * A;
  if (kok)
#pragma unroll
    for (int q = 0; q < 16; ++q) P[(long)((q & 3) + 8 * (q >> 2) + 4 * h) * A + k] = acc[q];
}

__global__ void k_tr_dwloc_fin(const float* __restrict__ G, const float* __restrict__ Kc, const float* __restrict__ bc,
                               int F, int A, int KW, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F * A) return;
  const int c = i / A, a = i % A;
  float v = bc[c] * G[31 * A + a];
  for (int tap = 0; tap < KW; ++tap) v += Kc[tap * F + c] * G[(long)tap * A + a];
  out[i] = v;
}

// prenet backward through dropout + ReLU: dz = (p > 0) ? 2·dp : 0   (p = relu(z)/0.5·keep)
__global__ void k_tr_prenet_bwd(const float* __restrict__ dp, long ld_dp, const float* __restrict__ p, long ld_p,
                                long M, int N, float* __restrict__ dz) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  const long m = i / N;
  const int n = (int)(i % N);
  dz[i] = p[m * ld_p + n] > 0.f ? 2.f * dp[m * ld_dp + n] : 0.f;
}

// d values of the attention context (context_t = align_t · values, attention.py:155-160), all rows in
// one launch: DVAL[b][j][d] = Σ_t ALIGN[b][j][t] · DCTX[t][b][d] on v_mfma_f32_16x16x4f32 (exact fp32
// products).  Work-group = (128 columns d, 64 rows j, row b), 8 waves: wave w owns column tile w over
// the 4 row tiles; t in LDS-staged chunks of 32 (8 k-steps).
constexpr int DV_JT = 64, DV_TC = 32;
__global__ __launch_bounds__(512) void k_tr_dval(const float* __restrict__ align, const float* __restrict__ dctx, int B,
                                                 int Tin, int T, int D, float* __restrict__ dval) {
  __shared__ float As[DV_JT][DV_TC + 1];
  __shared__ float Bs[DV_TC][128 + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g4 = lane >> 4;
  const int d0 = blockIdx.x * 128, j0 = blockIdx.y * DV_JT, b = blockIdx.z;
  const float* ab = align + (long)b * Tin * T;
  f32x4 acc[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the next chunk's operands are loaded into registers while the current chunk's products run
  constexpr int NA = DV_JT * DV_TC / 512, NB = DV_TC * 128 / 512;
  float pa[NA], pb[NB];
  auto load = [&](int t0) {
#pragma unroll
    for (int u = 0; u < NA; ++u) {  // coalesced over t
      const int e = tid + 512 * u, j = e / DV_TC, tt = e - j * DV_TC;
      pa[u] = (j0 + j < Tin && t0 + tt < T) ? ab[(long)(j0 + j) * T + t0 + tt] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {  // coalesced over d
      const int e = tid + 512 * u, tt = e >> 7, dd = e & 127;
      pb[u] = (t0 + tt < T && d0 + dd < D) ? dctx[((long)(t0 + tt) * B + b) * D + d0 + dd] : 0.f;
    }
  };
  load(0);
  for (int t0 = 0; t0 < T; t0 += DV_TC) {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int e = tid + 512 * u, j = e / DV_TC;
      As[j][e - j * DV_TC] = pa[u];
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = tid + 512 * u;
      Bs[e >> 7][e & 127] = pb[u];
    }
    __syncthreads();
    if (t0 + DV_TC < T) load(t0 + DV_TC);
#pragma unroll
    for (int ks = 0; ks < DV_TC / 4; ++ks) {
      const float bv = Bs[4 * ks + g4][16 * w + r16];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(As[16 * mt + r16][4 * ks + g4], bv, acc[mt], 0, 0, 0);
    }
    __syncthreads();
  }
  const int d = d0 + 16 * w + r16;
  if (d < D) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = j0 + 16 * mt + 4 * g4 + i;
        if (j < Tin) dval[((long)b * Tin + j) * D + d] = acc[mt][i];
      }
  }
}
__global__ void k_tr_mask_rows(const float* __restrict__ x, const int* __restrict__ lens, int B, int Tin, int D,
                               float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * Tin * D) return;
  const int j = (int)((i / D) % Tin), b = (int)(i / ((long)D * Tin));
  y[i] = j < lens[b] ? x[i] : 0.f;
}

// L2 regularisation (tacotron.py:865-867) of every regularised variable in ONE launch: block (x, y) takes
// variable y's [off, off + n) = seg[y] with the grid's x-stride, g += reg·w, partial Σ w²/2 -> part[64 y + x]
__global__ __launch_bounds__(256) void k_tr_reg(const float* __restrict__ w, float* __restrict__ g,
                                                const long2* __restrict__ seg, float reg, float* __restrict__ part) {
  __shared__ float s4[16];
  const long off = seg[blockIdx.y].x, n = seg[blockIdx.y].y;
  float acc = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = w[off + i];
    g[off + i] += reg * v;
    acc += 0.5f * v * v;
  }
  acc = block_sum(acc, s4);
  if (threadIdx.x == 0) part[64 * blockIdx.y + blockIdx.x] = acc;
}

// Zero-fill of up to TR_ZL_MAX device ranges in ONE launch (the step's state resets: a hipMemsetAsync costs
// ~6 us of launch each); 16-byte stores when a range's base is 16-byte aligned, else dwords
constexpr int TR_ZL_MAX = 16;
struct TrZeroList {
  void* p[TR_ZL_MAX];
  unsigned long long n[TR_ZL_MAX];  // bytes (multiples of 4)
  int count;
};
__global__ void k_tr_zero_many(TrZeroList z) {
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x,
                           stride = (unsigned long long)gridDim.x * blockDim.x;
  for (int i = 0; i < z.count; ++i) {
    if ((reinterpret_cast<uintptr_t>(z.p[i]) & 15) == 0) {
      uint4* q = reinterpret_cast<uint4*>(z.p[i]);
      const unsigned long long n16 = z.n[i] / 16;
      for (unsigned long long k = t; k < n16; k += stride) q[k] = make_uint4(0u, 0u, 0u, 0u);
      unsigned* w = reinterpret_cast<unsigned*>(z.p[i]);
      for (unsigned long long k = n16 * 4 + t; k < z.n[i] / 4; k += stride) w[k] = 0u;
    } else {
      unsigned* w = reinterpret_cast<unsigned*>(z.p[i]);
      for (unsigned long long k = t; k < z.n[i] / 4; k += stride) w[k] = 0u;
    }
  }
}
static void tr_zero_many(std::initializer_list<std::pair<void*, size_t>> l, hipStream_t s) {
  TrZeroList z{};
  unsigned long long tot = 0;
  for (const auto& e : l) {
    if (!e.first || !e.second) continue;
    if (z.count == TR_ZL_MAX) {  // full: flush
      hipLaunchKernelGGL(k_tr_zero_many, dim3((unsigned)std::min<unsigned long long>((tot / 16 + 255) / 256 + 1, 4096)),
                         dim3(256), 0, s, z);
      z.count = 0;
      tot = 0;
    }
    TT2_CHECK(e.second % 4 == 0, TT2_ERR_INVALID_ARG, "tr_zero_many: byte count % 4 != 0");
    z.p[z.count] = e.first;
    z.n[z.count++] = e.second;
    tot = std::max<unsigned long long>(tot, e.second);
  }
  if (z.count)
    hipLaunchKernelGGL(k_tr_zero_many, dim3((unsigned)std::min<unsigned long long>((tot / 16 + 255) / 256 + 1, 4096)),
                       dim3(256), 0, s, z);
  TT2_HIP(hipGetLastError());
}

// Σ g² partials per block: 16-byte loads when the gradient buffer is 16-byte aligned (a caller-bound
// buffer need not be), the tail by block 0
constexpr int TR_SUMSQ_BLOCKS = 1024;
__global__ __launch_bounds__(256) void k_tr_sumsq(const float* __restrict__ g, long n, float* __restrict__ part, int vec) {
  __shared__ float s4[16];
  float acc = 0.f;
  const long n4 = vec ? n / 4 : 0;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = g4[i];
    acc += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
  }
  for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += g[i] * g[i];
  acc = block_sum(acc, s4);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_tr_sum_final(const float* __restrict__ part, int nb, float scale,
                                                      float* __restrict__ out, int sq) {
  __shared__ double sd[256];
  double s = 0;
  for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
  s = block_sum256_d(s, sd);
  if (threadIdx.x != 0) return;
  out[0] = sq ? (float)sqrt(s) : (float)(s * scale);
}

// clip_by_global_norm(clip) + TF Adam (lr_t folded on the host)
// g[n] is the step's status word (k_tr_status; averaged over ranks with the gradients): nonzero when
// any rank's persistent forward failed, and then no rank applies the update
__global__ void k_tr_adam(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                          float* __restrict__ v, long n, const float* __restrict__ norm, float clip, float b1, float b2,
                          float eps, float lr_t) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || g[n] != 0.f) return;
  const float scale = clip > 0.f ? clip / fmaxf(norm[0], clip) : 1.f;
  const float gi = g[i] * scale;
  const float mi = b1 * m[i] + (1.f - b1) * gi;
  const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  w[i] -= lr_t * mi / (sqrtf(vi) + eps);
}

// ---- Postnet training (modules.py:474-497 in training mode) --------------------------------------
// column statistics over M rows: mode 0 sum(x); 1 sum((x - c)^2); per-split partials then final
__global__ __launch_bounds__(256) void k_pn_colstat_part(const float* __restrict__ x, long M, int N,
                                                         const float* __restrict__ ctr, int mode,
                                                         float* __restrict__ part) {
  __shared__ float red[256];
  const int TW = tr_tw(N), R = 256 / TW;
  const int cc = threadIdx.x % TW, r = threadIdx.x / TW;
  const int n = blockIdx.x * TW + cc;
  const int S = gridDim.y, sp = blockIdx.y;
  float acc = 0.f;
  if (n < N) {
    const float c0 = mode ? ctr[n] : 0.f;
#pragma unroll 4
    for (long m = (long)sp * R + r; m < M; m += (long)S * R) {
      const float v = x[m * N + n] - c0;
      acc += mode ? v * v : v;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (r == 0 && n < N) {
    float v = 0.f;
    for (int rr = 0; rr < R; ++rr) v += red[rr * TW + cc];
    part[(long)sp * N + n] = v;
  }
}
__global__ __launch_bounds__(TR_FIN) void k_pn_colstat_final(const float* __restrict__ part, int S, int N, float scale,
                                                             float* __restrict__ out) {
  __shared__ float red[32 * 33];
  const int n = blockIdx.x * 32 + (threadIdx.x & 31);
  const float tot = colsum_fin(part, S, N, n, n < N, red);
  if (threadIdx.x < 32 && n < N) out[n] = tot * scale;
}
// y = gamma (a - mean) rsqrt(var + eps) + beta, then dropout(0.5) with keep bits (or identity)
// planes (nullable): the next conv's padded bf16 input (gemm.h CX_* layout, rows b·T + t of y)
__device__ __forceinline__ void pn_plane_put(__bf16* planes, int T, long i, int C, float v) {
  const long m = i / C;
  const int c = (int)(i - m * C), b = (int)(m / T), t = (int)(m - (long)b * T);
  planes[(CX_G + (long)b * (T + 2 * CX_P) + CX_P + t) * C + c] = (__bf16)v;
}
__global__ void k_pn_bn_fwd(const float* __restrict__ a, long M, int C, const float* __restrict__ mean,
                            const float* __restrict__ var, const float* __restrict__ gamma,
                            const float* __restrict__ beta, float eps, const uint8_t* __restrict__ keep,
                            float* __restrict__ y, __bf16* __restrict__ planes = nullptr, int T = 1) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  float v = gamma[c] * (a[i] - mean[c]) * rsqrtf(var[c] + eps) + beta[c];
  if (keep) v = (v / 0.5f) * (float)keep[i];
  y[i] = v;
  if (planes) pn_plane_put(planes, T, i, C, v);
}
// BN backward sums over rows: S1 = sum dy, S2 = sum dy * xhat, with dy = dx_next * dropout
__global__ __launch_bounds__(256) void k_pn_bn_bwd_part(const float* __restrict__ dxn, const uint8_t* __restrict__ keep,
                                                        const float* __restrict__ a, long M, int C,
                                                        const float* __restrict__ mean, const float* __restrict__ var,
                                                        float eps, float* __restrict__ dy, float* __restrict__ part) {
  __shared__ float r1[256], r2[256];
  const int TW = tr_tw(C), R = 256 / TW;
  const int cc = threadIdx.x % TW, r = threadIdx.x / TW;
  const int c = blockIdx.x * TW + cc;
  const int S = gridDim.y, sp = blockIdx.y;
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    const float mu = mean[c], rs = rsqrtf(var[c] + eps);
#pragma unroll 4
    for (long m = (long)sp * R + r; m < M; m += (long)S * R) {
      const long i = m * C + c;
      float g = dxn[i];
      if (keep) g = g * 2.f * (float)keep[i];
      dy[i] = g;
      s1 += g;
      s2 += g * (a[i] - mu) * rs;
    }
  }
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  if (r == 0 && c < C) {
    float v1 = 0.f, v2 = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      v1 += r1[rr * TW + cc];
      v2 += r2[rr * TW + cc];
    }
    part[(long)sp * 2 * C + c] = v1;
    part[(long)sp * 2 * C + C + c] = v2;
  }
}
// finalize: d beta = S1, d gamma = S2 (written into the gradient slots)
__global__ __launch_bounds__(TR_FIN) void k_pn_bn_bwd_final(const float* __restrict__ part, int S, int C,
                                                            float* __restrict__ sums, float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta) {
  __shared__ float red[32 * 33];
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const float s1 = colsum_fin(part, S, 2L * C, c, c < C, red);
  const float s2 = colsum_fin(part + C, S, 2L * C, c, c < C, red);
  if (threadIdx.x >= 32 || c >= C) return;
  sums[c] = s1;
  sums[C + c] = s2;
  dbeta[c] = s1;
  dgamma[c] = s2;
}
// dz = [tanh'] gamma rstd (dy - S1/M - xhat S2/M)
__global__ void k_pn_bn_bwd_dz(const float* __restrict__ dy, const float* __restrict__ a, long M, int C,
                               const float* __restrict__ mean, const float* __restrict__ var, float eps,
                               const float* __restrict__ gamma, const float* __restrict__ sums, int tanh_act,
                               float* __restrict__ dz, __bf16* __restrict__ planes = nullptr, int T = 1) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  const float rs = rsqrtf(var[c] + eps);
  const float av = a[i];
  const float xh = (av - mean[c]) * rs;
  const float inv_m = 1.0f / (float)M;
  float g = gamma[c] * rs * (dy[i] - sums[c] * inv_m - xh * sums[C + c] * inv_m);
  if (tanh_act == 1) g *= 1.f - av * av;        // tanh (Postnet)
  else if (tanh_act == 2) g *= av > 0.f ? 1.f : 0.f;  // ReLU (encoder convolutions): av = relu output
  dz[i] = g;
  if (planes) pn_plane_put(planes, T, i, C, g);
}
// im2col^T of a conv1d input x(b, t, c) = x[b*xs_b + t*xs_t + c]:
// out[(tap*C + c) * ldo + b*T + t] = x(b, t + tap - pad, c) (0 outside [0, T))
__global__ void k_pn_im2col_t(const float* __restrict__ x, long xs_b, long xs_t, int B, int T, int C, int kw, int pad,
                              float* __restrict__ out, long ldo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long M = (long)B * T;
  if (i >= (long)kw * C * M) return;
  const long m = i % M;
  const long kc = i / M;
  const int c = (int)(kc % C), tap = (int)(kc / C);
  const int b = (int)(m / T), t = (int)(m % T);
  const int ts = t + tap - pad;
  out[kc * ldo + m] = (ts >= 0 && ts < T) ? x[(long)b * xs_b + (long)ts * xs_t + c] : 0.f;
}
// Wflip[(tap' * Cout + co) * Cin + ci] = W[((kw-1-tap') * Cin + ci) * Cout + co]  (conv1d input gradient)
__global__ void k_pn_flip(const float* __restrict__ w, int kw, int cin, int cout, float* __restrict__ wf) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)kw * cin * cout) return;
  const int ci = (int)(i % cin);
  const int co = (int)((i / cin) % cout);
  const int tp = (int)(i / ((long)cin * cout));
  wf[i] = w[((long)(kw - 1 - tp) * cin + ci) * cout + co];
}
// after loss: mel = clip(dec[t][b] + proj[b][t]) (tacotron.py:375-378); MSE partials; d proj
// inv = 1 / (MSE normaliser); tlen masks t >= lengths[b] (mask_decoder, MaskedMSE)
__global__ __launch_bounds__(256) void k_pn_after_loss(const float* __restrict__ FR, const float* __restrict__ prj,
                                                       const float* __restrict__ tg, int B, int T, int NM, int r,
                                                       int clip, float lo, float hi, float* __restrict__ dprj,
                                                       float* __restrict__ part, const int* __restrict__ tlen,
                                                       float inv) {
  __shared__ float s16[16];
  const long n = (long)B * T * NM;
  float sq = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % NM);
    const long bt = i / NM;
    const int t = (int)(bt % T), b = (int)(bt / T);
    const float x = FR[tr_frame_off(t, b, B, r, NM) + c] + prj[i];
    const float y = clip ? fminf(fmaxf(x, lo), hi) : x;
    const float d = (!tlen || t < tlen[b]) ? y - tg[i] : 0.f;
    sq += d * d;
    dprj[i] = (!clip || (x >= lo && x <= hi)) ? 2.f * d * inv : 0.f;
  }
  sq = block_sum(sq, s16);
  if (threadIdx.x == 0) part[blockIdx.x] = sq;
}
// dFR[t][b] += clipmask(frames) * (d mel + d postnet input)   (dec = clip(frames) feeds both)
__global__ void k_pn_add_ddec(const float* __restrict__ dprj, const float* __restrict__ dx0, const uint8_t* clipm,
                              int B, int T, int NM, int r, float* __restrict__ dFR) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * T * NM) return;
  const int c = (int)(i % NM);
  const long bt = i / NM;
  const int t = (int)(bt % T), b = (int)(bt / T);
  const long j = tr_frame_off(t, b, B, r, NM) + c;
  if (clipm[j]) dFR[j] += dprj[i] + dx0[i];
}
__global__ void k_pn_moving(float* __restrict__ mm, float* __restrict__ mv, const float* __restrict__ mean,
                            const float* __restrict__ var, int C, float momentum, const float* __restrict__ status) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C || status[0] != 0.f) return;
  mm[c] -= (mm[c] - mean[c]) * (1.f - momentum);
  mv[c] -= (mv[c] - var[c]) * (1.f - momentum);
}

// The step's status word behind the gradients (g[total]): 1 when the persistent forward of this step
// timed out in a hand-off or did not run every step (its control words), else 0.  It rides in the
// data-parallel tower mean with the gradients, so k_tr_adam / k_pn_moving on every rank skip an
// update that any rank's failed forward would have corrupted; tt2_train_losses then reports it.
__global__ void k_tr_status(const int* __restrict__ ctl, const int* __restrict__ ctl_bwd, int T,
                            float* __restrict__ status) {
  if (threadIdx.x == 0)
    status[0] = ((ctl && (ctl[0] != 0 || ctl[1] != T)) || (ctl_bwd && (ctl_bwd[0] != 0 || ctl_bwd[1] != T))) ? 1.f : 0.f;
}

// ---- host orchestration ----------------------------------------------------------------------
static inline unsigned nblk(long n, int t = 256) { return (unsigned)((n + t - 1) / t); }

static void tr_transpose(const float* src, long rows, long cols, long lds, float* dst, long ldd, hipStream_t s) {
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
  hipLaunchKernelGGL(k_tr_transpose, grid, dim3(256), 0, s, src, rows, cols, lds, dst, ldd);
}

static void tr_colsum(tt2_train_ctx* c, const float* in, long M, int N, long ld, float* out, hipStream_t s) {
  const int S = tr_splits(M, N, 64 * std::max<long>(4L * c->H, c->LX1));
  TT2_CHECK((size_t)S * N * sizeof(float) <= c->part.bytes, TT2_ERR_SHAPE_MISMATCH, "tr_colsum: partial buffer too small");
  hipLaunchKernelGGL(k_tr_colsum_part, dim3((N + tr_tw(N) - 1) / tr_tw(N), S), dim3(256), 0, s, in, M, N, ld,
                     c->part.as<float>());
  hipLaunchKernelGGL(k_tr_colsum_final, dim3((N + 31) / 32), dim3(TR_FIN), 0, s, c->part.as<float>(), S, N, out);
}

// per calling thread: the context a tt2_train_* call is driving (a call runs on one thread, so
// distinct contexts driven from different threads stay independent)
static thread_local DevBuf* g_tr_kpart = nullptr;  // split-K scratch (stream-ordered)
static thread_local int g_tr_prec = 0;             // GemmArgs::split16 (0 fp32, 2 bf16)
static thread_local tt2_train_ctx* g_tr_ctx = nullptr;  // bf16 BLAS scratch + handle of that context


// fp32 [rows][cols] (leading dimension ld) -> dense bf16 [rows][cols], round to nearest even (the
// same rounding the bf16 GEMM kernels apply when they stage operands)
__global__ void k_tr_to_bf16(const float* __restrict__ src, long rows, long cols, long ld, __bf16* __restrict__ dst) {
  const long n = rows * cols;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += (long)gridDim.x * blockDim.x * 4) {
    const long r = i / cols, cc = i % cols;
    if (cc + 3 < cols && ((r * ld + cc) & 3) == 0) {  // 16-byte aligned source quad
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + r * ld + cc);
      bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
      *reinterpret_cast<bf16x4*>(dst + i) = o;
    } else {
      for (int e = 0; e < 4 && i + e < n; ++e) {
        const long r2 = (i + e) / cols, c2 = (i + e) % cols;
        dst[i + e] = (__bf16)src[r2 * ld + c2];
      }
    }
  }
}

// The large plain products of the bf16 step (weight gradients over all T·B rows, the Postnet
// convolution gradients): C[M][N] = A[M][K]·B[K][N] on the hand-written 256 x 256 x 64 LDS-DMA bf16
// kernel (gemm.h gemm_bf16_kc: both operands rounded to bf16 into padded K-contiguous copies, B
// transposed on the way, K split over work-groups for the few-tile shapes, fp32 accumulation) --
// the same operand rounding as the per-step bf16 kernels.  Products below kTrBigMinFlops keep the
// per-step kernels' paths, except tall ones (>= 16k rows, N >= 256, K >= 64: e.g. d [h2 | ctx] =
// d frames · W_f^T over all T·B rows, bound by its output, which gemm_x3_kernel wrote at 0.6 TB/s).
static constexpr double kTrBigMinFlops = 2.0e10;
static bool tr_gemm_big(int M, int N, int K, const float* A, long lda, const float* Bw, long ldb, float* C, long ldc,
                        hipStream_t s) {
  tt2_train_ctx* c = g_tr_ctx;
  if (!c) return false;
  gemm_bf16_kc(M, N, K, A, lda, Bw, ldb, C, ldc, c->blasA, c->blasB, c->blasP, s);
  ++c->blas_calls;
  return true;
}

static void tr_gemm(int M, int N, int K, const float* A, long lda, const float* Bw, long ldb, float* C, long ldc,
                    hipStream_t s, const float* bias, const float* residual, long ldr, int act, const DevBuf* bt16,
                    long ldbt);

// Weight gradient C[M][N] = X^T·dG over K = T·B rows, X[K][M] (row stride ldx), dG[K][N]: the large
// ones straight from X on gemm_bf16_kc (its conversion pass transposes X), the rest through
// tr_transpose into TBUF and tr_gemm
static void tr_gemm_xtg(int M, int N, int K, const float* X, long ldx, const float* dG, long ldg, float* C, long ldc,
                        float* TBUF, hipStream_t s, const __bf16* dgt = nullptr) {
  tt2_train_ctx* c = g_tr_ctx;
  if (c && c->blas_on && g_tr_prec == 2 && 2.0 * M * (double)N * K >= kTrBigMinFlops) {
    // dgt: bf16(dG)^T already staged by the persistent backward (gemm_bf16_kc bt_pre)
    gemm_bf16_kc(M, N, K, X, ldx, dG, ldg, C, ldc, c->blasA, c->blasB, c->blasP, s, true, nullptr, dgt);
    ++c->blas_calls;
    return;
  }
  tr_transpose(X, K, M, ldx, TBUF, K, s);
  tr_gemm(M, N, K, TBUF, K, dG, ldg, C, ldc, s, nullptr, nullptr, 0, ACT_NONE, nullptr, 0);
}

static void tr_gemm(int M, int N, int K, const float* A, long lda, const float* Bw, long ldb, float* C, long ldc,
                    hipStream_t s, const float* bias = nullptr, const float* residual = nullptr, long ldr = 0,
                    int act = ACT_NONE, const DevBuf* bt16 = nullptr, long ldbt = 0) {
  if (g_tr_ctx && g_tr_ctx->blas_on && g_tr_prec == 2 && !bias && !residual && act == ACT_NONE &&
      (2.0 * M * (double)N * K >= kTrBigMinFlops || (M >= 16384 && N >= 256 && K >= 64)) &&
      tr_gemm_big(M, N, K, A, lda, Bw, ldb, C, ldc, s))
    return;
  GemmArgs g;
  if (g_tr_prec == 2 && bt16 && bt16->p && ldbt % 8 == 0) {  // weights pre-converted: B^T in bf16
    g.Bt16 = bt16->p;
    g.ldbt = ldbt;
  }
  if (g_tr_kpart) {
    g.kpart = g_tr_kpart->as<float>();
    g.kpart_floats = (long)(g_tr_kpart->bytes / sizeof(float));
  }
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.Bw = Bw; g.ldb = ldb; g.Cout = C; g.ldc = ldc;
  g.bias = bias; g.residual = residual; g.ldr = ldr; g.act = act;
  g.split16 = g_tr_prec;
  gemm(g, s);
}

// raw split-K product for a fused combine: partials [ks][M][N] in the context's kpart; returns ks
static int tr_gemm_raw(int M, int N, int K, const float* A, long lda, const float* Bw, long ldb, hipStream_t s,
                       const DevBuf* bt16 = nullptr, long ldbt = 0) {
  GemmArgs g;
  if (g_tr_prec == 2 && bt16 && bt16->p && ldbt % 8 == 0) {
    g.Bt16 = bt16->p;
    g.ldbt = ldbt;
  }
  g.kpart = g_tr_kpart->as<float>();
  g.kpart_floats = (long)(g_tr_kpart->bytes / sizeof(float));
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.Bw = Bw; g.ldb = ldb; g.Cout = nullptr; g.ldc = N;
  g.split16 = g_tr_prec;
  return gemm_raw(g, s);
}

static void tr_gemm_run(GemmArgs& g, hipStream_t s) {  // conv-mode products: same precision / split-K
  if (g_tr_kpart) {
    g.kpart = g_tr_kpart->as<float>();
    g.kpart_floats = (long)(g_tr_kpart->bytes / sizeof(float));
  }
  g.split16 = g_tr_prec;
  gemm(g, s);
}

static float* pvar(tt2_train_ctx* c, const std::string& n) { return c->params.as<float>() + c->vars[c->index.at(n)].off; }
static float* gvar(tt2_train_ctx* c, const std::string& n) { return c->grads + c->vars[c->index.at(n)].off; }

static const char* TP = "Tacotron_model/inference/";
static std::string vn(const char* s) { return std::string(TP) + s; }
#define LAV(x) vn("decoder/Location_Sensitive_Attention/" x)
#define L1V(x) vn("decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/" x)
#define L2V(x) vn("decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/" x)
#define FPV(x) vn("decoder/linear_transform_projection/projection_linear_transform_projection/" x)
#define SPV(x) vn("decoder/stop_token_projection/projection_stop_token_projection/" x)
#define PRV(i, x) vn((std::string("decoder/decoder_prenet/dense_") + std::to_string(i) + "/" x).c_str())

// TT2_REDZONE: name of one of the context's buffers (redzone reports)
static std::string tr_bufname(const void* owner, const DevBuf* b) {
  const tt2_train_ctx* c = static_cast<const tt2_train_ctx*>(owner);
#define TT2_NM(x) if (b == &c->x) return #x;
#define TT2_NMA(x, n) for (int i_ = 0; i_ < (n); ++i_) if (b == &c->x[i_]) return std::string(#x "[") + std::to_string(i_) + "]";
  TT2_NM(params) TT2_NM(grads_own) TT2_NM(adam_m) TT2_NM(adam_v) TT2_NM(K1T) TT2_NM(K2T) TT2_NM(WqT) TT2_NM(WfT)
  TT2_NM(WsT) TT2_NM(WmT) TT2_NM(Wp2T) TT2_NM(values) TT2_NM(keys) TT2_NM(X1) TT2_NM(X2) TT2_NM(PIN) TT2_NM(G1)
  TT2_NM(G2) TT2_NM(C1) TT2_NM(C2) TT2_NM(CN1) TT2_NM(CN2) TT2_NM(Q) TT2_NM(ALIGN) TT2_NM(CUM) TT2_NM(P1)
  TT2_NM(XIN) TT2_NM(FR) TT2_NM(ST) TT2_NM(dFR) TT2_NM(dST) TT2_NM(dPIN) TT2_NM(dX1) TT2_NM(dX2) TT2_NM(dG1)
  TT2_NM(dG2) TT2_NM(DC1) TT2_NM(DC2) TT2_NM(R1) TT2_NM(R2) TT2_NM(DQ) TT2_NM(DCTX) TT2_NM(DKEYS) TT2_NM(DCUM)
  TT2_NM(dV) TT2_NM(dBA) TT2_NM(dKC) TT2_NM(dBC) TT2_NM(DVAL) TT2_NM(DMEM) TT2_NM(dZ) TT2_NM(dPre) TT2_NM(TBUF)
  TT2_NM(part) TT2_NM(red) TT2_NM(kpart) TT2_NM(TH) TT2_NM(E) TT2_NM(DF) TT2_NM(PQ) TT2_NM(FALL) TT2_NM(ALN)
  TT2_NM(blasA) TT2_NM(blasB) TT2_NM(blasP) TT2_NM(hK1) TT2_NM(hK1T) TT2_NM(hK2) TT2_NM(hK2T) TT2_NM(hWq) TT2_NM(hWqT) TT2_NM(X1h) TT2_NM(X2h) TT2_NM(dGh) TT2_NM(tK1T) TT2_NM(tK2T) TT2_NM(tWq) TT2_NM(tK2) TT2_NM(tK1)
  TT2_NMA(PA, 8) TT2_NMA(PX, 9) TT2_NM(BNM) TT2_NM(BNV) TT2_NM(PPRJ) TT2_NM(dPP) TT2_NM(DYb) TT2_NM(DZb)
  TT2_NM(dPXa) TT2_NM(dPXb) TT2_NM(WFLIP) TT2_NM(PWT) TT2_NM(CLIPM) TT2_NM(pn_part) TT2_NM(fEX) TT2_NMA(fEA, 8)
  TT2_NMA(fEY, 9) TT2_NM(fXP) TT2_NM(fGZ) TT2_NM(fGA) TT2_NM(fCN) TT2_NM(fCS) TT2_NM(fHS) TT2_NM(fENC)
  TT2_NM(fTWf) TT2_NM(fTWb) TT2_NM(fHSh) TT2_NM(fDZh) TT2_NM(fMEM) TT2_NM(fSTY) TT2_NM(fDSTY) TT2_NM(fDZ) TT2_NM(fDHC) TT2_NM(fDCC) TT2_NM(fDHP) TT2_NM(fdXP)
  TT2_NM(fdA) TT2_NM(fdB) TT2_NM(fLWxT) TT2_NM(fLWhT) TT2_NMA(fXG, 2) TT2_NMA(fGR, 2) TT2_NMA(fGU, 2)
  TT2_NMA(fGCC, 2) TT2_NMA(fGRH, 2) TT2_NMA(fHG, 2) TT2_NMA(fREF, 2) TT2_NM(fGG) TT2_NM(fGC) TT2_NM(fFBUF)
  TT2_NM(fDY) TT2_NM(fDY2) TT2_NM(fDZc) TT2_NM(fGq) TT2_NM(fGkk) TT2_NM(fGv) TT2_NM(fGnv) TT2_NM(fGbb)
  TT2_NM(fGsum) TT2_NM(fdREF) TT2_NM(fDZD) TT2_NM(fDH) TT2_NM(fDHA) TT2_NM(fDRH) TT2_NM(fDCP) TT2_NM(fDGP)
  TT2_NM(fDXG) TT2_NM(fWT) TT2_NM(fBN) TT2_NM(fpart)
  for (int r = 0; r < 2; ++r)
    for (int i = 0; i < 6; ++i) {
      if (b == &c->fRA[r][i]) return "fRA[" + std::to_string(r) + "][" + std::to_string(i) + "]";
      if (b == &c->fRY[r][i]) return "fRY[" + std::to_string(r) + "][" + std::to_string(i) + "]";
    }
#undef TT2_NM
#undef TT2_NMA
  return "";
}
// TT2_REDZONE: fail the call naming every buffer a kernel of this phase wrote past
static void tr_redzones(tt2_train_ctx* c, const char* phase) {
  if (!redzone_on()) return;
  const std::string r = redzone_check(phase, tr_bufname, c);
  TT2_CHECK(r.empty(), TT2_ERR_HIP, "redzone violation: " + r);
}

static void tr_front_build_vars(tt2_train_ctx* c,
                                const std::function<void(const std::string&, std::vector<int64_t>, bool)>& add);

static void tr_build_vars(tt2_train_ctx* c) {
  const int D = c->D, A = c->A, F = c->F, KW = c->KW, P = c->P, H = c->H, NM = c->NM;
  auto add = [&](const std::string& n, std::vector<int64_t> sh, bool reg) {
    TrVar v;
    v.name = n;
    v.shape = sh;
    v.n = 1;
    for (auto d : sh) v.n *= d;
    v.off = c->total;
    v.reg = reg;
    c->total += (v.n + 63) / 64 * 64;  // 256-byte aligned segments
    c->index[n] = (int)c->vars.size();
    c->vars.push_back(v);
  };
  // order and regularisation mask: oracle/train_ref.py train_var_names() / regularized()
  add(vn("memory_layer/kernel"), {D, A}, true);
  add(vn("decoder/query_layer/kernel"), {H, A}, true);
  add(LAV("location_features_convolution/kernel"), {KW, 1, F}, true);
  add(LAV("location_features_convolution/bias"), {F}, false);
  add(LAV("location_features_layer/kernel"), {F, A}, true);
  add(LAV("attention_variable_projection"), {A}, false);
  add(LAV("attention_bias"), {A}, false);
  add(PRV(1, "kernel"), {NM, P}, true);
  add(PRV(1, "bias"), {P}, false);
  add(PRV(2, "kernel"), {P, P}, true);
  add(PRV(2, "bias"), {P}, false);
  add(L1V("kernel"), {P + D + H, 4 * H}, false);
  add(L1V("bias"), {4 * H}, false);
  add(L2V("kernel"), {2 * H, 4 * H}, false);
  add(L2V("bias"), {4 * H}, false);
  add(FPV("kernel"), {H + D, (int64_t)NM * c->R}, false);  // num_mels * r (tacotron.py:322)
  add(FPV("bias"), {(int64_t)NM * c->R}, false);
  add(SPV("kernel"), {H + D, c->R}, false);                   // shape = r (tacotron.py:324)
  add(SPV("bias"), {c->R}, false);
  if (c->cfg.frontend) tr_front_build_vars(c, add);
  if (!c->cfg.postnet) return;
  // Postnet (oracle/train_ref.py postnet_var_names / postnet_stat_names); moving statistics are
  // non-trainable slots of the same table (zero gradient -> Adam leaves them alone)
  for (int i = 1; i <= c->PL; ++i) {
    const std::string sc = vn("postnet_convolutions/conv_layer_") + std::to_string(i) + "_postnet_convolutions/";
    const int cin = i == 1 ? NM : c->PC;
    add(sc + "conv1d/kernel", {c->PK, cin, c->PC}, true);
    add(sc + "conv1d/bias", {c->PC}, false);
    add(sc + "batch_normalization/gamma", {c->PC}, true);
    add(sc + "batch_normalization/beta", {c->PC}, true);
    add(sc + "batch_normalization/moving_mean", {c->PC}, false);
    add(sc + "batch_normalization/moving_variance", {c->PC}, false);
  }
  add(vn("postnet_projection/projection_postnet_projection/kernel"), {c->PC, NM}, false);
  add(vn("postnet_projection/projection_postnet_projection/bias"), {NM}, false);
}

static std::string pn_scope(int i) {
  return vn("postnet_convolutions/conv_layer_") + std::to_string(i) + "_postnet_convolutions/";
}

static void tr_front_alloc(tt2_train_ctx* c);

static void tr_alloc(tt2_train_ctx* c) {
  const long B = c->B, T = c->Tm, Tin = c->Tin, D = c->D, H = c->H, P = c->P, A = c->A, F = c->F, KW = c->KW,
             NM = c->NM, LX1 = c->LX1;
  const long TB = T * B;
  auto f = [](DevBuf& d, long n) { d.alloc(sizeof(float) * (size_t)std::max<long>(n, 1)); };
  f(c->params, c->total); f(c->grads_own, c->total + 1);  // + the status word (k_tr_status)
  f(c->adam_m, c->total); f(c->adam_v, c->total);
  c->grads = c->grads_own.as<float>();
  f(c->K1T, 4 * H * LX1); f(c->K2T, 4 * H * 2 * H); f(c->WqT, A * H); f(c->WfT, NM * c->R * (H + D)); f(c->WsT, c->R * (H + D));
  f(c->WmT, A * D); f(c->Wp2T, P * P);
  f(c->values, B * Tin * D); f(c->keys, B * Tin * A);
  f(c->X1, (T + 1) * B * LX1); f(c->X2, (T + 1) * B * 2 * H); f(c->PIN, TB * (H + D));
  f(c->G1, TB * 4 * H); f(c->G2, TB * 4 * H); f(c->C1, (T + 1) * B * H); f(c->C2, (T + 1) * B * H);
  f(c->CN1, TB * H); f(c->CN2, TB * H); f(c->Q, TB * A); f(c->ALIGN, B * Tin * T); f(c->CUM, (T + 1) * B * Tin);
  f(c->P1, TB * P); f(c->XIN, TB * NM); f(c->FR, TB * NM); f(c->ST, TB);
  f(c->dFR, TB * NM); f(c->dST, TB); f(c->dPIN, TB * (H + D)); f(c->dX1, (T + 1) * B * LX1);
  f(c->dX2, (T + 1) * B * 2 * H); f(c->dG1, TB * 4 * H); f(c->dG2, TB * 4 * H); f(c->DC1, B * H); f(c->DC2, B * H);
  f(c->R1, B * LX1); f(c->R2, B * 2 * H); f(c->DQ, TB * A); f(c->DCTX, TB * D);
  const long NT = (Tin + TR_JT - 1) / TR_JT;
  f(c->DKEYS, B * Tin * A); f(c->DCUM, B * Tin); f(c->dV, B * NT * A); f(c->dBA, B * NT * A);
  f(c->dKC, B * NT * KW * F); f(c->dBC, B * NT * F); f(c->FALL, TB * Tin * F); f(c->ALN, TB * Tin);
  f(c->TH, TB * Tin * A); f(c->E, B * Tin); f(c->DF, B * Tin * F); f(c->PQ, B * NT * A); f(c->DVAL, B * Tin * D); f(c->DMEM, B * Tin * D);
  f(c->dZ, TB * P); f(c->dPre, TB * P);
  f(c->DF2, 2 * B * Tin * F); f(c->DCUM2, 2 * B * Tin); f(c->PQ2, 2 * B * NT * A); f(c->SC2, 2 * B * 4); f(c->DWG, 32 * A);
  f(c->DWGP, B * NT * 32 * A);
  f(c->W1T, P * NM); f(c->sDZ, B * P); f(c->sDP, B * P); f(c->sDX, B * NM); c->TLEN.alloc(sizeof(int) * (size_t)B);
  const long tmax = std::max({TB * LX1, TB * (H + D), TB * 2 * H, B * Tin * D, TB * P, TB * NM, TB * Tin * F,
                              // Postnet im2col^T: K·cin rows per position, cin = num_mels for layer 1
                              c->cfg.postnet ? TB * (long)c->PK * std::max<long>(c->PC, NM) : 0L});
  f(c->TBUF, tmax);
  f(c->part, 64 * std::max<long>(4 * H, LX1) + 4096);
  f(c->red, 64);  // loss / norm slots
  if (c->cfg.precision) {
    auto h = [](DevBuf& d, long n) { d.alloc(2 * (size_t)std::max<long>(n, 1)); };
    h(c->hK1, LX1 * 4 * H); h(c->hK1T, LX1 * 4 * H); h(c->hK2, 8 * H * H); h(c->hK2T, 8 * H * H);
    h(c->hWq, H * A); h(c->hWqT, H * A);
    const long Bp = (B + 31) & ~31L;  // TF-layout shadows: row blocks of 32
    h(c->X1h, (T + 1) * Bp * LX1); h(c->X2h, (T + 1) * Bp * 2 * H); h(c->dGh, 2 * Bp * 4 * H);
    h(c->tK1T, LX1 * 4 * H); h(c->tK2T, 8 * H * H); h(c->tWq, H * A); h(c->tK2, 8 * H * H);
    h(c->tK1, ((LX1 + 31) / 32 * 32) * 4 * H);
    // padded bf16 operand copies of the large products (tr_gemm_big -> gemm_bf16_kc): the largest
    // weight gradients over all T·B rows -- LSTM-1 [LX1 x TB]·[TB x 4H], the Postnet convs
    // [K·cin x TB]·[TB x PC]; rows to 256, K to the split's 64-multiple (<= TB + 64·257), and the
    // split-K partials (ks·Mp·Np <= 256 tiles of 256 x 256)
    const long pcin = c->cfg.postnet ? (long)c->PK * std::max<long>(c->PC, NM) : 0L;
    const long Kpm = TB + 64L * 257, r256 = 255;
    h(c->blasA, ((std::max({LX1, 2 * H, pcin}) + r256) & ~r256) * Kpm);
    h(c->blasB, ((std::max<long>(4 * H, c->cfg.postnet ? c->PC : 0) + r256) & ~r256) * Kpm);
    f(c->blasP, 256L * 256 * 256);
  }
  f(c->kpart, 4L << 20);
  if (c->cfg.frontend) tr_front_alloc(c);
  if (c->cfg.postnet) {
    const long PC = c->PC, PK = c->PK;
    for (int i = 0; i < c->PL; ++i) f(c->PA[i], TB * PC);
    for (int i = 1; i <= c->PL; ++i) f(c->PX[i], TB * PC);
    f(c->BNM, c->PL * PC); f(c->BNV, c->PL * PC); f(c->PPRJ, TB * NM); f(c->dPP, TB * NM);
    // layer inputs' gradients: PC channels, num_mels for the first layer (may exceed PC)
    f(c->DYb, TB * PC); f(c->DZb, TB * PC); f(c->dPXa, TB * std::max(PC, NM)); f(c->dPXb, TB * std::max(PC, NM));
    f(c->WFLIP, PK * std::max(PC, NM) * PC);  // flipped kernels: layer 1's are [PK][num_mels][PC]
    f(c->PWT, NM * PC); f(c->pn_part, 64 * 2 * PC + 1024);
    {
      const char* e = std::getenv("TT2_PN_PLANES");  // 0: the implicit-im2col gemm_x3_kernel convs
      c->pn_planes = (!e || std::atoi(e) != 0) && c->cfg.precision && PC % 64 == 0 && (PK & 1) && PK <= 2 * CX_P + 1;
    }
    if (c->pn_planes) {
      const long W = std::max<long>(PC, NM), Wr = (W + 255) / 256 * 256;
      c->pnPl.alloc((size_t)cx_rows(c->B, (int)(TB / c->B)) * PC * 2);
      c->pnWt.alloc((size_t)Wr * PK * W * 2);
    }
    c->CLIPM.alloc((size_t)TB * NM);
    if (c->R > 1) f(c->FRT, TB * NM);
  }
}

// Postnet forward (training-mode BN + dropout) + after loss + backward; adds d decoder_output into
// dFR (through the frame clip).  Runs between the decoder forward and the decoder backward.  T = frames
// (decoder steps · r).
static void tr_postnet(tt2_train_ctx* c, const float* tg, const uint8_t* pnm, int T, hipStream_t s) {
  const int B = c->B, NM = c->NM, C = c->PC, KW = c->PK, L = c->PL;
  const long M = (long)B * T;
  const int pad = (KW - 1) / 2;
  const float eps = c->cfg.bn_eps;
  float* red = c->red.as<float>();
  float* part = c->pn_part.as<float>();
  float* sums = part + 64L * 2 * C;
  float* TBUF = c->TBUF.as<float>();
  const int S = tr_splits(M, C, 64L * C);
  const unsigned CT = (unsigned)((C + tr_tw(C) - 1) / tr_tw(C));
  auto colstat = [&](const float* x, const float* ctr, int mode, float* out) {
    hipLaunchKernelGGL(k_pn_colstat_part, dim3(CT, S), dim3(256), 0, s, x, M, C, ctr, mode, part);
    hipLaunchKernelGGL(k_pn_colstat_final, dim3((C + 31) / 32), dim3(TR_FIN), 0, s, part, S, C, 1.0f / (float)M, out);
  };
  auto conv_in = [&](int i, GemmArgs& g) {  // layer i's input as an implicit-im2col conv1d operand
    if (i == 0) {  // clipped decoder frames, time-major [T][B][NM] (r > 1: the FRT copy)
      g.A = c->R > 1 ? c->FRT.as<float>() : c->FR.as<float>(); g.C = NM; g.xs_b = NM; g.xs_t = (long)B * NM;
    } else {
      g.A = c->PX[i].as<float>(); g.C = C; g.xs_b = (long)T * C; g.xs_t = C;
    }
  };
  const bool planes = c->pn_planes && g_tr_prec == 2;
  __bf16* pl = reinterpret_cast<__bf16*>(c->pnPl.p);
  __bf16* wt = reinterpret_cast<__bf16*>(c->pnWt.p);
  if (planes && (c->pn_pl_B != B || c->pn_pl_T != T)) {  // pad and guard rows stay zero from here on
    TT2_HIP(hipMemsetAsync(c->pnPl.p, 0, (size_t)cx_rows(B, T) * C * 2, s));
    c->pn_pl_B = B;
    c->pn_pl_T = T;
  }
  const int Cr = (C + 255) / 256 * 256;
  if (c->R > 1)
    hipLaunchKernelGGL(k_tr_frames_tm, dim3(nblk(M * NM)), dim3(256), 0, s, c->FR.as<float>(), B, T, NM, c->R,
                       c->FRT.as<float>());
  for (int i = 0; i < L; ++i) {
    const std::string sc = pn_scope(i + 1);
    if (planes && i > 0) {  // layer i's input planes were written by layer i-1's BN forward
      kc_transpose_bf16(pvar(c, sc + "conv1d/kernel"), KW * C, C, C, wt, KW * C, Cr, s);
      conv_bf16_planes(pl, C, B, T, KW, wt, (long)KW * C, C, pvar(c, sc + "conv1d/bias"),
                       i < L - 1 ? ACT_TANH : ACT_NONE, c->PA[i].as<float>(), C, s);
    } else {
      GemmArgs g;
      g.a_mode = A_CONV1D; g.M = (int)M; g.N = C; g.T = T; g.kw = KW; g.pad = pad;
      conv_in(i, g);
      g.K = KW * g.C;
      g.Bw = pvar(c, sc + "conv1d/kernel"); g.ldb = C; g.Cout = c->PA[i].as<float>(); g.ldc = C;
      g.bias = pvar(c, sc + "conv1d/bias"); g.act = i < L - 1 ? ACT_TANH : ACT_NONE;
      tr_gemm_run(g, s);
    }
    float* mean = c->BNM.as<float>() + (long)i * C;
    float* var = c->BNV.as<float>() + (long)i * C;
    colstat(c->PA[i].as<float>(), nullptr, 0, mean);
    colstat(c->PA[i].as<float>(), mean, 1, var);
    hipLaunchKernelGGL(k_pn_bn_fwd, dim3(nblk(M * C)), dim3(256), 0, s, c->PA[i].as<float>(), M, C, mean, var,
                       pvar(c, sc + "batch_normalization/gamma"), pvar(c, sc + "batch_normalization/beta"), eps,
                       pnm ? pnm + (long)i * M * C : nullptr, c->PX[i + 1].as<float>(),
                       planes && i < L - 1 ? pl : nullptr, T);
  }
  const std::string pp = vn("postnet_projection/projection_postnet_projection/");
  tr_gemm((int)M, NM, C, c->PX[L].as<float>(), C, pvar(c, pp + "kernel"), NM, c->PPRJ.as<float>(), NM, s,
          pvar(c, pp + "bias"));
  const int* tlen = c->cfg.mask_decoder ? c->TLEN.as<int>() : nullptr;
  const double nmse = c->cfg.mask_decoder ? (double)c->tlen_sum * NM : (double)M * NM;
  hipLaunchKernelGGL(k_pn_after_loss, dim3(256), dim3(256), 0, s, c->FR.as<float>(), c->PPRJ.as<float>(), tg, B, T,
                     NM, c->R, c->cfg.clip_outputs, c->cfg.clip_lo, c->cfg.clip_hi, c->dPP.as<float>(), c->part.as<float>(),
                     tlen, (float)(1.0 / nmse));
  hipLaunchKernelGGL(k_tr_sum_final, dim3(1), dim3(256), 0, s, c->part.as<float>(), 256, (float)(1.0 / nmse),
                     red + 4, 0);
  // backward: projection
  tr_transpose(c->PX[L].as<float>(), M, C, C, TBUF, M, s);
  tr_gemm(C, NM, (int)M, TBUF, M, c->dPP.as<float>(), NM, gvar(c, pp + "kernel"), NM, s);
  tr_colsum(c, c->dPP.as<float>(), M, NM, NM, gvar(c, pp + "bias"), s);
  tr_transpose(pvar(c, pp + "kernel"), C, NM, NM, c->PWT.as<float>(), C, s);
  float* dxn = c->dPXa.as<float>();
  float* dxo = c->dPXb.as<float>();
  tr_gemm((int)M, C, NM, c->dPP.as<float>(), NM, c->PWT.as<float>(), C, dxn, C, s);
  for (int i = L - 1; i >= 0; --i) {
    const std::string sc = pn_scope(i + 1);
    const float* mean = c->BNM.as<float>() + (long)i * C;
    const float* var = c->BNV.as<float>() + (long)i * C;
    hipLaunchKernelGGL(k_pn_bn_bwd_part, dim3(CT, S), dim3(256), 0, s, dxn,
                       pnm ? pnm + (long)i * M * C : nullptr, c->PA[i].as<float>(), M, C, mean, var, eps,
                       c->DYb.as<float>(), part);
    hipLaunchKernelGGL(k_pn_bn_bwd_final, dim3((C + 31) / 32), dim3(TR_FIN), 0, s, part, S, C, sums,
                       gvar(c, sc + "batch_normalization/gamma"), gvar(c, sc + "batch_normalization/beta"));
    hipLaunchKernelGGL(k_pn_bn_bwd_dz, dim3(nblk(M * C)), dim3(256), 0, s, c->DYb.as<float>(), c->PA[i].as<float>(),
                       M, C, mean, var, eps, pvar(c, sc + "batch_normalization/gamma"), sums, i < L - 1 ? 1 : 0,
                       c->DZb.as<float>(), planes ? pl : nullptr, T);
    tr_colsum(c, c->DZb.as<float>(), M, C, C, gvar(c, sc + "conv1d/bias"), s);
    const int cin = i == 0 ? NM : C;
    {
      GemmArgs gi;
      conv_in(i, gi);
      if (c->blas_on && g_tr_prec == 2 && 2.0 * KW * cin * (double)C * M >= kTrBigMinFlops) {
        KcConvA cv;  // im2colᵀ gathered straight into gemm_bf16_kc's bf16 operand copy
        cv.x = gi.A; cv.xs_b = gi.xs_b; cv.xs_t = gi.xs_t; cv.B = B; cv.T = T; cv.C = cin; cv.kw = KW; cv.pad = pad;
        gemm_bf16_kc(KW * cin, C, (int)M, nullptr, 0, c->DZb.as<float>(), C, gvar(c, sc + "conv1d/kernel"), C,
                     c->blasA, c->blasB, c->blasP, s, false, &cv);
        ++c->blas_calls;
      } else {
        hipLaunchKernelGGL(k_pn_im2col_t, dim3(nblk((long)KW * cin * M)), dim3(256), 0, s, gi.A, gi.xs_b, gi.xs_t, B,
                           T, cin, KW, pad, TBUF, M);
        tr_gemm(KW * cin, C, (int)M, TBUF, M, c->DZb.as<float>(), C, gvar(c, sc + "conv1d/kernel"), C, s);
      }
    }
    hipLaunchKernelGGL(k_pn_flip, dim3(nblk((long)KW * cin * C)), dim3(256), 0, s, pvar(c, sc + "conv1d/kernel"), KW,
                       cin, C, c->WFLIP.as<float>());
    if (planes) {  // input gradient: conv of the dz planes with the flipped kernel (pad KW-1-pad = pad)
      kc_transpose_bf16(c->WFLIP.as<float>(), KW * C, cin, cin, wt, KW * C, (cin + 255) / 256 * 256, s);
      conv_bf16_planes(pl, C, B, T, KW, wt, (long)KW * C, cin, nullptr, ACT_NONE, dxo, cin, s);
    } else {
      GemmArgs g;
      g.a_mode = A_CONV1D; g.M = (int)M; g.N = cin; g.T = T; g.kw = KW; g.pad = KW - 1 - pad;
      g.A = c->DZb.as<float>(); g.C = C; g.xs_b = (long)T * C; g.xs_t = C; g.K = KW * C;
      g.Bw = c->WFLIP.as<float>(); g.ldb = cin; g.Cout = dxo; g.ldc = cin;
      tr_gemm_run(g, s);
    }
    std::swap(dxn, dxo);
  }
  hipLaunchKernelGGL(k_pn_add_ddec, dim3(nblk(M * NM)), dim3(256), 0, s, c->dPP.as<float>(), dxn,
                     c->CLIPM.as<uint8_t>(), B, T, NM, c->R, c->dFR.as<float>());
  c->pn_ran = true;
}

// any step of the next T fed its own previous frame (tt2_train_set_teacher_forcing)
static bool tr_has_free_steps(const tt2_train_ctx* c, int T) {
  if (c->feed.empty()) return false;
  TT2_CHECK((int)c->feed.size() >= T, TT2_ERR_SHAPE_MISMATCH,
            "teacher-forcing draw shorter than T_out (tt2_train_set_teacher_forcing)");
  for (int t = 1; t < T; ++t)
    if (!c->feed[t]) return true;
  return false;
}

// forward + losses + backward for one batch; grads complete (incl. L2) on return (stream order)
// Y[m][n] += u[m]·v[n] over M x N (N % 4 == 0, 16-byte rows): the stop projection's d input
__global__ void k_tr_rank1_add(float* __restrict__ Y, long ld, const float* __restrict__ u, const float* __restrict__ v,
                               long M, int N) {
  const int n4 = N >> 2;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < M * n4; i += (long)gridDim.x * blockDim.x) {
    const long m = i / n4;
    const int c = (int)(i - m * n4) * 4;
    f32x4* y = reinterpret_cast<f32x4*>(Y + m * ld + c);
    const f32x4 w = *reinterpret_cast<const f32x4*>(v + c);
    *y += u[m] * w;
  }
}

// d W_loc from the cumulative alignments (k_tr_dwloc_cum) instead of the stored location features:
// the forward then skips FALL (TT2_TR_DWLOC_CUM=0: FALL + k_tr_dwloc)
static bool tr_dwloc_cum_ok(const tt2_train_ctx* c) {
  static const bool env = [] {
    const char* e = std::getenv("TT2_TR_DWLOC_CUM");
    return !(e && e[0] == '0');
  }();
  return env && c->KW <= 31 && c->F <= 32 && c->A <= 128;
}

// Persistent forward (train_persist.hip): fork widths (H 1024, prenet 256, memory 1024, attention 128
// x 32 filters), B <= 64, T_in <= TP_TMAX, bf16 operands with the bf16 values copy, every step
// teacher-forced (a step fed its own frame needs the frame projection inside the loop).
static bool tr_persist_fits(const tt2_train_ctx* c, int Tin, bool free_run, bool values16) {
  return c->tp_on && !free_run && values16 && !c->cfg.smoothing && c->B <= 64 && Tin <= TP_TMAX && c->H == TP_H && c->P == TP_P &&
         c->D == TP_D && c->A == TP_A && c->F == TP_F && c->KW == TP_KWMAX && c->LX1 == TP_LX1;
}

static void tr_persist_forward(tt2_train_ctx* c, const TrAtt& at, const uint8_t* zm, int Tin, int T, hipStream_t s) {
  const size_t xb = 2ul * 64 * 1024 * sizeof(__bf16);  // two parities of [64][1024] bf16
  auto grow = [](DevBuf& d, size_t n) {
    if (d.bytes < n) d.alloc(n);
  };
  for (DevBuf* d : {&c->tpCX, &c->tpH1X, &c->tpZ1X, &c->tpH2X, &c->tpZ2X}) grow(*d, xb);
  grow(c->tpEX, 2ul * 64 * 4 * TP_TMAX * sizeof(unsigned long long));
  grow(c->tpCtl, sizeof(unsigned) * (3ul * TP_NREP * TP_NB + 16));
  grow(c->tpPre, (size_t)T * 64 * TP_P * sizeof(__bf16));
  grow(c->tpKWT, sizeof(float) * TP_A * 32);
  if (!c->tp_ctl_host) TT2_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->tp_ctl_host), 4 * sizeof(int)));
  // rows >= B of the exchange buffers stay zero (they are A-operand padding); the flags and the
  // granules restart their tags at 1 every launch
  for (DevBuf* d : {&c->tpCX, &c->tpH1X, &c->tpZ1X, &c->tpH2X, &c->tpZ2X, &c->tpEX, &c->tpCtl})
    TT2_HIP(hipMemsetAsync(d->p, 0, d->bytes, s));
  tp_prenet_rows(c->X1.as<float>(), c->LX1, c->B, T, c->tpPre.as<__bf16>(), s);
  tp_prepare(at.Kc, at.bc, at.Wl, c->tpKWT.as<float>(), s);
  TpArgs a{};
  a.B = c->B; a.T = T; a.Tin = Tin; a.KW = c->KW; a.z = c->cfg.zoneout;
  a.K1T = c->hK1T.as<__bf16>(); a.K2T = c->hK2T.as<__bf16>(); a.Wq = c->hWq.as<__bf16>();
  a.b1 = pvar(c, L1V("bias")); a.b2 = pvar(c, L2V("bias"));
  a.Kc = at.Kc; a.bc = at.bc; a.Wl = at.Wl; a.va = at.va; a.ba = at.ba; a.KWT = c->tpKWT.as<float>();
  a.keys = at.keys; a.values16 = at.values16; a.lens = at.lens; a.zm = zm; a.preh = c->tpPre.as<__bf16>();
  a.X1 = c->X1.as<float>(); a.X2 = c->X2.as<float>(); a.PIN = c->PIN.as<float>();
  a.G1 = c->G1.as<float>(); a.G2 = c->G2.as<float>(); a.CN1 = c->CN1.as<float>(); a.CN2 = c->CN2.as<float>();
  a.C1 = c->C1.as<float>(); a.C2 = c->C2.as<float>(); a.ALIGN = at.ALIGN; a.CUM = at.CUM; a.TH = at.TH;
  a.FALL = at.FALL; a.ALN = at.ALN;
  // the persistent backward's packed unit operands (train_persist.h TpArgs::BPK), when it will run
  a.BPK = nullptr;
  if (c->tb_on && Tin <= TB_TMAX) {
    grow(c->tbPK, (size_t)T * TP_NB * 4 * TP_NT * 4 * sizeof(float));
    a.BPK = c->tbPK.as<float>();
  }
  a.CX = c->tpCX.as<__bf16>(); a.H1X = c->tpH1X.as<__bf16>(); a.Z1X = c->tpZ1X.as<__bf16>();
  a.H2X = c->tpH2X.as<__bf16>(); a.Z2X = c->tpZ2X.as<__bf16>();
  a.EX = c->tpEX.as<unsigned long long>();
  a.flags = c->tpCtl.as<unsigned>();
  a.ctl = reinterpret_cast<int*>(a.flags + 3 * TP_NREP * TP_NB);
  // TT2_TP_STAMP=<step>: stage stamps of that step -> TT2_TP_STAMP_FILE (int64 [256][32], diagnostic)
  const char* st = std::getenv("TT2_TP_STAMP");
  a.stamp_step = st ? std::atoi(st) : -1;
  {  // TT2_TP_OC: placement of the forward's off-chain products (A/B; k_tr_persist)
    const char* e = std::getenv("TT2_TP_OC");
    a.oc_mode = e ? std::atoi(e) : 1;  // mode 1 measured 69.9 against 70.45 ms/step (mode 0)
  }
  a.stamps = nullptr;
  if (st) {
    grow(c->tpStamps, sizeof(long long) * TP_NB * 32);
    TT2_HIP(hipMemsetAsync(c->tpStamps.p, 0, c->tpStamps.bytes, s));
    a.stamps = c->tpStamps.as<long long>();
  }
  tp_launch(a, s);
  c->tp_ctl_dev = a.ctl;
  // TT2_TP_FORCE_FAIL=1 (test hook): mark this launch's control word as a timed-out hand-off in phase
  // 0, as a stalled launch would, to exercise the status word and the skipped update
  if (const char* ff = std::getenv("TT2_TP_FORCE_FAIL"))
    if (ff[0] == '1') TT2_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(a.ctl), 1, 1, s));
  if (!tr_dwloc_cum_ok(c)) tp_location_features(at.CUM, at.Kc, at.bc, c->B, T, Tin, at.FALL, s);
  if (st) {
    std::vector<long long> h((size_t)TP_NB * 32);
    TT2_HIP(hipMemcpyAsync(h.data(), a.stamps, h.size() * sizeof(long long), hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
    const char* fn = std::getenv("TT2_TP_STAMP_FILE");
    if (FILE* f = std::fopen(fn ? fn : "tp_stamps.bin", "wb")) {
      std::fwrite(h.data(), sizeof(long long), h.size(), f);
      std::fclose(f);
    }
  }
  TT2_HIP(hipMemcpyAsync(c->tp_ctl_host, a.ctl, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
  c->tp_check = true;
}

// Control words of the last persistent forward (after the stream has passed it): a timed-out
// hand-off or a launch that did not run every step fails the read-back that follows the step.
static void tr_persist_check(tt2_train_ctx* c) {
  if (!c->tp_check && !c->tb_check) return;
  TT2_HIP(hipStreamSynchronize(c->last_stream));
  const bool fwd = c->tp_check, bwd = c->tb_check;
  c->tp_check = c->tb_check = false;
  if (fwd) {
    const int ph = c->tp_ctl_host[0], steps = c->tp_ctl_host[1];
    TT2_CHECK(ph == 0, TT2_ERR_HIP,
              "persistent training forward: a hand-off wait timed out (phase " + std::to_string(ph - 1) +
                  "); TT2_TR_PERSIST=0 runs the per-step launches");
    TT2_CHECK(steps == c->T_last, TT2_ERR_STATE, "persistent training forward did not complete every step");
  }
  if (bwd) {
    const int ph = c->tp_ctl_host[2], steps = c->tp_ctl_host[3];
    TT2_CHECK(ph == 0, TT2_ERR_HIP,
              "persistent training backward: a hand-off wait timed out (phase " + std::to_string(ph - 1) +
                  "); TT2_TR_PERSIST_BWD=0 runs the per-step launches");
    TT2_CHECK(steps == c->T_last, TT2_ERR_STATE, "persistent training backward did not complete every step");
  }
}

// Persistent backward of the decoder loop (train_bwd_persist.hip): the fork geometry of the
// persistent forward, bf16 fused step, every step teacher-forced, softmax attention
static void tr_persist_backward(tt2_train_ctx* c, const TrAtt& at, const uint8_t* zm, int Tin, int T, int NT,
                                hipStream_t s) {
  const int B = c->B;
  auto grow = [](DevBuf& d, size_t n) {
    if (d.bytes < n) d.alloc(n);
  };
  const size_t xg = 2ul * 64 * 4 * TP_H * sizeof(__bf16);
  grow(c->tbG1X, xg);
  grow(c->tbG2X, xg);
  grow(c->tbP1X, 2ul * TB_NKB * 64 * TB_NOUT * sizeof(float));
  grow(c->tbP2X, 2ul * TB_NKB * 64 * TB_NOUT * sizeof(float));
  grow(c->tbQX, 2ul * 64 * TP_A * sizeof(__bf16));
  grow(c->tbW1F, (size_t)TP_NB * 4 * 16 * 64 * 8 * sizeof(__bf16));
  grow(c->tpEX, 2ul * 64 * 4 * TP_TMAX * sizeof(unsigned long long));
  grow(c->tbCtl, sizeof(unsigned) * ((size_t)TB_NPH * TP_NREP * TP_NB + 16));
  if (!c->tp_ctl_host) TT2_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->tp_ctl_host), 4 * sizeof(int)));
  // rows >= B of the dG exchange rows stay zero (A-operand padding); tags restart at 1 every launch
  tr_zero_many({{c->tbG1X.p, c->tbG1X.bytes}, {c->tbG2X.p, c->tbG2X.bytes}, {c->tbQX.p, c->tbQX.bytes},
                {c->tpEX.p, c->tpEX.bytes}, {c->tbCtl.p, c->tbCtl.bytes}, {c->DWGP.p, c->DWGP.bytes}},
               s);
  TbArgs a{};
  a.B = B; a.T = T; a.Tin = Tin; a.NT = NT; a.z = c->cfg.zoneout;
  a.K1T = c->hK1T.as<__bf16>(); a.K2T = c->hK2T.as<__bf16>(); a.Wq = c->hWq.as<__bf16>();
  a.va = at.va; a.KWT = c->tpKWT.as<float>(); a.values16 = at.values16; a.lens = at.lens;
  a.ALN = at.ALN; a.CUM = at.CUM; a.TH = at.TH;
  TT2_CHECK(c->tbPK.bytes >= (size_t)T * TP_NB * 4 * TP_NT * 4 * sizeof(float), TT2_ERR_STATE,
            "persistent backward: the forward did not pack the unit operands");
  a.BPK = c->tbPK.as<float>(); a.dPIN = c->dPIN.as<float>();
  // bf16(dG)^T in the layout the weight-gradient GEMMs stage (B = 64: the K index t·64 + row is t·B + b),
  // when both products' K split keeps Kp = T·B (no padding columns to clear)
  a.DGT1 = a.DGT2 = nullptr;
  a.DGR1 = nullptr;
  a.dgt_ld = 0;
  c->tb_dgt = c->tb_dgr = false;
  {
    long np1, kp1, np2, kp2;
    gemm_bf16_kc_bt_dims(c->LX1, 4 * TP_H, T * B, &np1, &kp1);
    gemm_bf16_kc_bt_dims(2 * TP_H, 4 * TP_H, T * B, &np2, &kp2);
    const char* e = std::getenv("TT2_TB_DGT");
    if (B == 64 && c->blas_on && g_tr_prec == 2 && np1 == 4 * TP_H && np2 == 4 * TP_H && kp1 == (long)T * B &&
        kp2 == kp1 && !(e && e[0] == '0')) {
      grow(c->tbDGT1, (size_t)4 * TP_H * kp1 * sizeof(__bf16));
      grow(c->tbDGT2, (size_t)4 * TP_H * kp1 * sizeof(__bf16));
      a.DGT1 = c->tbDGT1.as<__bf16>();
      a.DGT2 = c->tbDGT2.as<__bf16>();
      a.dgt_ld = kp1;
      c->tb_dgt = true;
      // the d X1 product's A staging is bf16(dG1) row-major when its K split keeps Kp = 4H
      long np3, kp3;
      gemm_bf16_kc_bt_dims(T * B, TP_P, 4 * TP_H, &np3, &kp3);
      if (kp3 == 4 * TP_H) {
        grow(c->tbDGR1, (size_t)T * B * 4 * TP_H * sizeof(__bf16));
        a.DGR1 = c->tbDGR1.as<__bf16>();
        c->tb_dgr = true;
      }
    }
  }
  a.dG1 = c->dG1.as<float>(); a.dG2 = c->dG2.as<float>(); a.DQ = c->DQ.as<float>(); a.DCTX = c->DCTX.as<float>();
  a.DKEYS = c->DKEYS.as<float>(); a.dV = c->dV.as<float>(); a.dBA = c->dBA.as<float>(); a.DWGP = c->DWGP.as<float>();
  a.G1X = c->tbG1X.as<__bf16>(); a.G2X = c->tbG2X.as<__bf16>(); a.P1X = c->tbP1X.as<float>();
  a.P2X = c->tbP2X.as<float>(); a.DQX = c->tbQX.as<__bf16>(); a.EX = c->tpEX.as<unsigned long long>();
  a.W1F = c->tbW1F.as<__bf16>();
  a.flags = c->tbCtl.as<unsigned>();
  a.ctl = reinterpret_cast<int*>(a.flags + (size_t)TB_NPH * TP_NREP * TP_NB);
  // TT2_TB_STAMP=<step>: stage stamps of that step -> TT2_TB_STAMP_FILE (int64 [256][32], diagnostic)
  const char* st = std::getenv("TT2_TB_STAMP");
  a.stamp_step = st ? std::atoi(st) : -1;
  a.stamps = nullptr;
  if (st) {
    grow(c->tpStamps, sizeof(long long) * TP_NB * 32);
    TT2_HIP(hipMemsetAsync(c->tpStamps.p, 0, c->tpStamps.bytes, s));
    a.stamps = c->tpStamps.as<long long>();
  }
  tb_launch(a, s);
  c->tb_ctl_dev = a.ctl;
  if (st) {
    std::vector<long long> h((size_t)TP_NB * 32);
    TT2_HIP(hipMemcpyAsync(h.data(), a.stamps, h.size() * sizeof(long long), hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
    const char* fn = std::getenv("TT2_TB_STAMP_FILE");
    if (FILE* f = std::fopen(fn ? fn : "tb_stamps.bin", "wb")) {
      std::fwrite(h.data(), sizeof(long long), h.size(), f);
      std::fclose(f);
    }
  }
  TT2_HIP(hipMemcpyAsync(c->tp_ctl_host + 2, a.ctl, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
  c->tb_check = true;
}

static void tr_write_status(tt2_train_ctx* c, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_status, dim3(1), dim3(64), 0, s, c->tp_last ? c->tp_ctl_dev : nullptr,
                     c->tb_last ? c->tb_ctl_dev : nullptr, c->T_last,
                     c->grads + c->total);
}

static void tr_forward_backward(tt2_train_ctx* c, const float* mem, const int* lens, const float* tg, const float* stg,
                                const uint8_t* pm, const uint8_t* zm, const uint8_t* pnm, int Tin, int Tf,
                                hipStream_t s) {
  const int B = c->B, D = c->D, H = c->H, P = c->P, A = c->A, F = c->F, KW = c->KW, NM = c->NM, LX1 = c->LX1;
  // Tf frames = T decoder steps of R frames each (outputs_per_step; the feeder pads targets to a
  // multiple of r, feeder.py:283-310)
  const int R = c->R;
  TT2_CHECK(Tf % R == 0, TT2_ERR_SHAPE_MISMATCH, "T_out must be a multiple of outputs_per_step");
  const int T = Tf / R;
  const int NR = NM * R;  // frame projection width num_mels * r
  const long TB = (long)T * B;
  const float z = c->cfg.zoneout;
  // tacotron.py:56-57 (the reference raises RuntimeError) and the MaskedMSE shape assert
  // (modules.py:549-550: mask length = max(lengths) must equal T_out)
  TT2_CHECK(!c->cfg.mask_decoder || c->has_tlen, TT2_ERR_STATE,
            "Model set to mask paddings but no targets lengths provided for the mask! "
            "(tt2_train_set_target_lengths)");
  // (sequence_mask rounds max(lengths) up to a multiple of r, modules.py:523-530)
  TT2_CHECK(!c->cfg.mask_decoder || (c->tlen_max + R - 1) / R * R == Tf, TT2_ERR_SHAPE_MISMATCH,
            "mask_decoder: max(target lengths) rounded up to outputs_per_step must equal T_out");
  c->T_last = T;
  c->Tf_last = Tf;
  c->Tin_last = Tin;
  g_tr_kpart = &c->kpart;
  g_tr_prec = c->cfg.precision ? 2 : 0;
  g_tr_ctx = c;
  // weight transposes for the backward products
  tr_transpose(pvar(c, L1V("kernel")), LX1, 4 * H, 4 * H, c->K1T.as<float>(), LX1, s);
  tr_transpose(pvar(c, L2V("kernel")), 2 * H, 4 * H, 4 * H, c->K2T.as<float>(), 2 * H, s);
  tr_transpose(pvar(c, vn("decoder/query_layer/kernel")), H, A, A, c->WqT.as<float>(), H, s);
  tr_transpose(pvar(c, FPV("kernel")), H + D, NR, NR, c->WfT.as<float>(), H + D, s);
  tr_transpose(pvar(c, SPV("kernel")), H + D, R, R, c->WsT.as<float>(), H + D, s);
  tr_transpose(pvar(c, vn("memory_layer/kernel")), D, A, A, c->WmT.as<float>(), D, s);
  tr_transpose(pvar(c, PRV(2, "kernel")), P, P, P, c->Wp2T.as<float>(), P, s);
  if (c->cfg.precision) {
    auto cv = [&](const float* src, long n, DevBuf& d) {
      hipLaunchKernelGGL(k_tr_to_bf16, dim3(nblk(n)), dim3(256), 0, s, src, n, d.as<__bf16>());
    };
    cv(pvar(c, L1V("kernel")), (long)LX1 * 4 * H, c->hK1);
    cv(c->K1T.as<float>(), (long)LX1 * 4 * H, c->hK1T);
    cv(pvar(c, L2V("kernel")), 8L * H * H, c->hK2);
    cv(c->K2T.as<float>(), 8L * H * H, c->hK2T);
    cv(pvar(c, vn("decoder/query_layer/kernel")), (long)H * A, c->hWq);
    cv(c->WqT.as<float>(), (long)H * A, c->hWqT);
  }
  TT2_HIP(hipMemsetAsync(c->grads, 0, sizeof(float) * (c->total + 1), s));
  TT2_HIP(hipMemsetAsync(c->red.p, 0xFF, 4 * sizeof(float), s));  // NaN until this call's losses land

  // ---- forward ----
  float* X1 = c->X1.as<float>();
  float* X2 = c->X2.as<float>();
  float* PIN = c->PIN.as<float>();
  tr_zero_many({{X1, sizeof(float) * (size_t)B * LX1},  // slot 0: ctx_{-1} = h_{-1} = 0
                {X2, sizeof(float) * (size_t)B * 2 * H}, {c->C1.p, sizeof(float) * (size_t)B * H},
                {c->C2.p, sizeof(float) * (size_t)B * H}, {c->CUM.p, sizeof(float) * (size_t)B * Tin}},
               s);
  hipLaunchKernelGGL(k_tr_inputs, dim3(nblk(TB * NM)), dim3(256), 0, s, tg, B, T, NM, R, c->XIN.as<float>());
  hipLaunchKernelGGL(k_tr_values, dim3(nblk((long)B * Tin * D)), dim3(256), 0, s, mem, lens, B, Tin, D,
                     c->values.as<float>());
  tr_gemm(B * Tin, A, D, c->values.as<float>(), D, pvar(c, vn("memory_layer/kernel")), A, c->keys.as<float>(), A, s);
  // prenet over all steps at once (teacher-forced inputs are known up front)
  tr_gemm((int)TB, P, NM, c->XIN.as<float>(), NM, pvar(c, PRV(1, "kernel")), P, c->P1.as<float>(), P, s,
          pvar(c, PRV(1, "bias")), nullptr, 0, ACT_RELU);
  hipLaunchKernelGGL(k_tr_prenet_mask, dim3(nblk(TB * P)), dim3(256), 0, s, c->P1.as<float>(), (long)P, pm, 0, T, B, P);
  tr_gemm((int)TB, P, P, c->P1.as<float>(), P, pvar(c, PRV(2, "kernel")), P, X1, LX1, s, pvar(c, PRV(2, "bias")),
          nullptr, 0, ACT_RELU);
  hipLaunchKernelGGL(k_tr_prenet_mask, dim3(nblk(TB * P)), dim3(256), 0, s, X1, (long)LX1, pm, 1, T, B, P);
  // fused per-step products (k_tr_fused: product + consumer epilogue in one launch, forward and
  // backward) on bf16 shadows of their input rows; TT2_TR_FUSED=0 keeps the split-K products +
  // combines (A/B)
  const char* fe = std::getenv("TT2_TR_FUSED");
  const bool fused_env = !(fe && fe[0] == '0');
  const bool fused = fused_env && g_tr_prec == 2 && B <= 64 && H % 32 == 0 && LX1 % 128 == 0 && A % 128 == 0;
  __bf16* X1h = fused ? c->X1h.as<__bf16>() : nullptr;
  __bf16* X2h = fused ? c->X2h.as<__bf16>() : nullptr;
  const long Bp = (B + 31) & ~31L;  // rows per step of the TF-layout shadows
  if (fused) {
    TT2_HIP(hipMemsetAsync(X1h, 0, 2 * (size_t)Bp * LX1, s));      // slot 0: ctx_{-1} = h_{-1} = 0
    TT2_HIP(hipMemsetAsync(X2h, 0, 2 * (size_t)Bp * 2 * H, s));
    TT2_HIP(hipMemsetAsync(c->dGh.p, 0, c->dGh.bytes, s));          // padding rows stay 0
    hipLaunchKernelGGL(k_tr_rows_bf16, dim3(2048), dim3(256), 0, s, X1, (long)LX1, TB, P, B, LX1, X1h);
    // the fused products' weights in TF layout, column-group order (once per step: the weights change
    // with every apply)
    auto tw = [&](const DevBuf& src, int N, int K, int ncg, int mode, DevBuf& dst) {
      hipLaunchKernelGGL(k_tr_tf_weights, dim3(2048), dim3(256), 0, s, src.as<__bf16>(), N, K, ncg, mode, H,
                         dst.as<__bf16>());
    };
    tw(c->hK1T, 4 * H, LX1, H / 8, TF_FWD, c->tK1T);
    tw(c->hK2T, 4 * H, 2 * H, H / 8, TF_FWD, c->tK2T);
    tw(c->hWq, H, A, H / 32, TF_BWD_H, c->tWq);
    tw(c->hK2, 2 * H, 4 * H, H / 16, TF_BWD_S, c->tK2);
    tw(c->hK1, LX1, 4 * H, (LX1 + 31) / 32, TF_PLAIN, c->tK1);
    TT2_HIP(hipGetLastError());
  }

  TrAtt at{};
  at.B = B; at.Tin = Tin; at.T = T; at.A = A; at.F = F; at.KW = KW; at.D = D; at.H = H; at.P = P;
  at.lens = lens; at.keys = c->keys.as<float>(); at.values = c->values.as<float>(); at.Q = c->Q.as<float>();
  at.values16 = nullptr;
  if (g_tr_prec == 2 && c->values16_on && (D & 3) == 0) {  // bf16 copy of this step's values (once per step)
    if (c->values16.bytes < (size_t)B * Tin * D * 2) c->values16.alloc((size_t)B * Tin * D * 2);  // grow only
    hipLaunchKernelGGL(k_tr_to_bf16, dim3(2048), dim3(256), 0, s, c->values.as<float>(), (long)B * Tin, (long)D, (long)D,
                       c->values16.as<__bf16>());
    TT2_HIP(hipGetLastError());
    at.values16 = c->values16.as<__bf16>();
  }
  at.Kc = pvar(c, LAV("location_features_convolution/kernel"));
  at.bc = pvar(c, LAV("location_features_convolution/bias"));
  at.Wl = pvar(c, LAV("location_features_layer/kernel"));
  at.va = pvar(c, LAV("attention_variable_projection"));
  at.ba = pvar(c, LAV("attention_bias"));
  at.ALIGN = c->ALIGN.as<float>(); at.CUM = c->CUM.as<float>(); at.PIN = PIN; at.X1 = X1;
  at.X1h = fused ? c->X1h.as<__bf16>() : nullptr;
  at.dPIN = c->dPIN.as<float>(); at.dX1 = c->dX1.as<float>(); at.DCTX = c->DCTX.as<float>(); at.DQ = c->DQ.as<float>();
  at.DKEYS = c->DKEYS.as<float>(); at.DCUM = c->DCUM.as<float>(); at.dV = c->dV.as<float>(); at.dBA = c->dBA.as<float>();
  at.dKC = c->dKC.as<float>(); at.dBC = c->dBC.as<float>();
  at.FALL = c->FALL.as<float>(); at.ALN = c->ALN.as<float>();
  at.TH = c->TH.as<float>(); at.E = c->E.as<float>(); at.DF = c->DF.as<float>();
  at.PQ = c->PQ.as<float>();
  at.smooth = c->cfg.smoothing ? 1 : 0;
  if (at.smooth) {
    if (c->SS.bytes < sizeof(float) * (size_t)T * B) c->SS.alloc(sizeof(float) * (size_t)T * B);
    at.SS = c->SS.as<float>();
  }
  const int NT = (Tin + TR_JT - 1) / TR_JT;
  at.nt = NT;
  const dim3 att_grid(NT, B);
  static const bool tr_e2 = [] {  // TT2_TR_E2=0: the 1024-thread energy kernel (A/B)
    const char* e = std::getenv("TT2_TR_E2");
    return !(e && e[0] == '0');
  }();
  const unsigned bh = nblk((long)B * H);

  // teacher-forcing draw (TacoTrainingHelper.next_inputs, helpers.py:122-133): a step fed its own
  // previous frame re-runs the prenet for its B rows from that frame (unclipped frame projection,
  // Architecture_wrappers.py:258-263); XIN / P1 / X1 then hold what the step actually consumed
  const bool free_run = tr_has_free_steps(c, T);
  if (free_run) tr_transpose(pvar(c, PRV(1, "kernel")), NM, P, P, c->W1T.as<float>(), NM, s);
  // the whole teacher-forced loop as one persistent launch when the shapes are the fork's
  c->tp_last = fused && tr_persist_fits(c, Tin, free_run, at.values16 != nullptr);
  if (c->tp_last) tr_persist_forward(c, at, zm, Tin, T, s);
  for (int t = 0; t < (c->tp_last ? 0 : T); ++t) {
    const long s1 = (long)t * B;
    if (free_run && t > 0 && !c->feed[t]) {
      float* xin = c->XIN.as<float>() + s1 * NM;
      float* p1 = c->P1.as<float>() + s1 * P;
      // the last of step t-1's r frames (outputs[:, -output_dim:], helpers.py:129)
      tr_gemm(B, NM, H + D, PIN + (s1 - B) * (H + D), H + D, pvar(c, FPV("kernel")) + (R - 1) * NM, NR, xin, NM, s,
              pvar(c, FPV("bias")) + (R - 1) * NM);
      tr_gemm(B, P, NM, xin, NM, pvar(c, PRV(1, "kernel")), P, p1, P, s, pvar(c, PRV(1, "bias")), nullptr, 0,
              ACT_RELU);
      hipLaunchKernelGGL(k_tr_prenet_mask, dim3(nblk((long)B * P)), dim3(256), 0, s, p1, (long)P,
                         pm + (long)t * 2 * B * P, 0, 1, B, P);
      tr_gemm(B, P, P, p1, P, pvar(c, PRV(2, "kernel")), P, X1 + s1 * LX1, LX1, s, pvar(c, PRV(2, "bias")), nullptr,
              0, ACT_RELU);
      hipLaunchKernelGGL(k_tr_prenet_mask, dim3(nblk((long)B * P)), dim3(256), 0, s, X1 + s1 * LX1, (long)LX1,
                         pm + (long)t * 2 * B * P, 1, 1, B, P);
      if (fused)
        hipLaunchKernelGGL(k_tr_rows_bf16, dim3(nblk((long)B * P)), dim3(256), 0, s, X1 + s1 * LX1, (long)LX1, (long)B,
                           P, B, LX1, X1h + t * Bp * LX1);
    }
    if (fused) {  // LSTM-1 and LSTM-2: product + bias + cell + zoneout in one launch each
      TrFused f{};
      f.Ah = X1h + t * Bp * LX1; f.Wt = c->tK1T.as<__bf16>(); f.K = LX1; f.bias = pvar(c, L1V("bias"));
      f.c_prev = c->C1.as<float>() + s1 * H; f.hz_prev = X1 + s1 * LX1 + P + D; f.ld_hz_prev = LX1;
      f.zm = zm; f.t = t; f.layer = 0; f.B = B; f.H = H; f.z = z;
      f.G = c->G1.as<float>() + s1 * 4 * H; f.cn = c->CN1.as<float>() + s1 * H; f.c_out = c->C1.as<float>() + (s1 + B) * H;
      f.h_out = X2 + s1 * 2 * H; f.ld_h = 2 * H; f.hz_out = X1 + (s1 + B) * LX1 + P + D; f.ld_hz = LX1;
      f.h_out_h = X2h + t * Bp * 2 * H; f.ld_h_h = 2 * H; f.h_col0 = 0;
      f.hz_out_h = X1h + (t + 1) * Bp * LX1; f.ld_hz_h = LX1; f.hz_col0 = P + D;
      hipLaunchKernelGGL(k_tr_fused<TF_FWD>, dim3(2 * H / TLG_U), dim3(TLG_NT), 0, s, f);
      TrFused f2{};
      f2.Ah = X2h + t * Bp * 2 * H; f2.Wt = c->tK2T.as<__bf16>(); f2.K = 2 * H; f2.bias = pvar(c, L2V("bias"));
      f2.c_prev = c->C2.as<float>() + s1 * H; f2.hz_prev = X2 + s1 * 2 * H + H; f2.ld_hz_prev = 2 * H;
      f2.zm = zm; f2.t = t; f2.layer = 1; f2.B = B; f2.H = H; f2.z = z;
      f2.G = c->G2.as<float>() + s1 * 4 * H; f2.cn = c->CN2.as<float>() + s1 * H;
      f2.c_out = c->C2.as<float>() + (s1 + B) * H;
      f2.h_out = PIN + s1 * (H + D); f2.ld_h = H + D; f2.hz_out = X2 + (s1 + B) * 2 * H + H; f2.ld_hz = 2 * H;
      f2.hz_out_h = X2h + (t + 1) * Bp * 2 * H; f2.ld_hz_h = 2 * H; f2.hz_col0 = H;
      hipLaunchKernelGGL(k_tr_fused<TF_FWD>, dim3(2 * H / TLG_U), dim3(TLG_NT), 0, s, f2);
    } else {
      // LSTM-1: raw split-K product, combine + bias + cell + zoneout fused in k_tr_lstm_fwd
      const int k1 = tr_gemm_raw(B, 4 * H, LX1, X1 + s1 * LX1, LX1, pvar(c, L1V("kernel")), 4 * H, s, &c->hK1T, LX1);
      TrLstmFwd l1{};
      l1.G = c->G1.as<float>() + s1 * 4 * H; l1.part = c->kpart.as<float>(); l1.ks = k1; l1.bias = pvar(c, L1V("bias"));
      l1.c_prev = c->C1.as<float>() + s1 * H; l1.hz_prev = X1 + s1 * LX1 + P + D; l1.ld_hz_prev = LX1;
      l1.zm = zm; l1.t = t; l1.layer = 0; l1.B = B; l1.H = H; l1.z = z;
      l1.cn = c->CN1.as<float>() + s1 * H; l1.c_out = c->C1.as<float>() + (s1 + B) * H;
      l1.h_out = X2 + s1 * 2 * H; l1.ld_h = 2 * H; l1.hz_out = X1 + (s1 + B) * LX1 + P + D; l1.ld_hz = LX1;
      hipLaunchKernelGGL(k_tr_lstm_fwd, dim3(bh), dim3(256), 0, s, l1);
      const int k2 = tr_gemm_raw(B, 4 * H, 2 * H, X2 + s1 * 2 * H, 2 * H, pvar(c, L2V("kernel")), 4 * H, s, &c->hK2T,
                                 2 * H);
      TrLstmFwd l2{};
      l2.G = c->G2.as<float>() + s1 * 4 * H; l2.part = c->kpart.as<float>(); l2.ks = k2; l2.bias = pvar(c, L2V("bias"));
      l2.c_prev = c->C2.as<float>() + s1 * H; l2.hz_prev = X2 + s1 * 2 * H + H; l2.ld_hz_prev = 2 * H;
      l2.zm = zm; l2.t = t; l2.layer = 1; l2.B = B; l2.H = H; l2.z = z;
      l2.cn = c->CN2.as<float>() + s1 * H; l2.c_out = c->C2.as<float>() + (s1 + B) * H;
      l2.h_out = PIN + s1 * (H + D); l2.ld_h = H + D; l2.hz_out = X2 + (s1 + B) * 2 * H + H; l2.ld_hz = 2 * H;
      hipLaunchKernelGGL(k_tr_lstm_fwd, dim3(bh), dim3(256), 0, s, l2);
    }
    at.t = t;
    if (A <= 128 && tr_e2) {  // query as raw split-K partials, combined inside the energy kernel
      at.qks = tr_gemm_raw(B, A, H, PIN + s1 * (H + D), H + D, pvar(c, vn("decoder/query_layer/kernel")), A, s,
                           &c->hWqT, H);
      at.qpart = c->kpart.as<float>();
      hipLaunchKernelGGL(k_tr_att_energy2, att_grid, dim3(TR_E2T), 0, s, at);
      at.qpart = nullptr;
    } else {
      tr_gemm(B, A, H, PIN + s1 * (H + D), H + D, pvar(c, vn("decoder/query_layer/kernel")), A,
              c->Q.as<float>() + s1 * A, A, s, nullptr, nullptr, 0, ACT_NONE, &c->hWqT, H);
      hipLaunchKernelGGL(k_tr_att_energy, att_grid, dim3(TR_AT), 0, s, at);
    }
    hipLaunchKernelGGL(k_tr_ctx, dim3((D + 63) / 64, B), dim3(256), sizeof(float) * Tin, s, at);
  }
  tr_gemm((int)TB, NR, H + D, PIN, H + D, pvar(c, FPV("kernel")), NR, c->FR.as<float>(), NR, s, pvar(c, FPV("bias")));
  tr_gemm((int)TB, R, H + D, PIN, H + D, pvar(c, SPV("kernel")), R, c->ST.as<float>(), R, s, pvar(c, SPV("bias")));
  float* red = c->red.as<float>();
  const int* tlen = c->cfg.mask_decoder ? c->TLEN.as<int>() : nullptr;
  const long nmse = c->cfg.mask_decoder ? c->tlen_sum * NM : TB * NR;
  hipLaunchKernelGGL(k_tr_loss, dim3(256), dim3(256), 0, s, c->FR.as<float>(), c->ST.as<float>(), tg, stg, B, Tf, NM,
                     R, c->cfg.clip_outputs, c->cfg.clip_lo, c->cfg.clip_hi, c->dFR.as<float>(), c->dST.as<float>(),
                     c->part.as<float>(), c->cfg.postnet ? c->CLIPM.as<uint8_t>() : nullptr, tlen,
                     (float)(1.0 / (double)nmse), c->cfg.pos_weight);
  hipLaunchKernelGGL(k_tr_loss_final, dim3(1), dim3(256), 0, s, c->part.as<float>(), 256, nmse, tlen ? 0L : TB * R,
                     red);
  if (tlen) hipLaunchKernelGGL(k_tr_div, dim3(nblk(TB * R)), dim3(256), 0, s, c->dST.as<float>(), TB * R, red + 5);
  c->pn_ran = false;
  if (c->cfg.postnet) tr_postnet(c, tg, pnm, Tf, s);

  // ---- backward ----
  float* dPIN = c->dPIN.as<float>();
  float* dX1 = c->dX1.as<float>();
  float* dX2 = c->dX2.as<float>();
  tr_gemm((int)TB, H + D, NR, c->dFR.as<float>(), NR, c->WfT.as<float>(), H + D, dPIN, H + D, s);
  // + dST·W_s^T: a rank-1 update, streamed (as a K = 1 GEMM with the residual it took 0.69 ms); rank r
  // for r > 1
  if (R > 1)
    tr_gemm((int)TB, H + D, R, c->dST.as<float>(), R, c->WsT.as<float>(), H + D, dPIN, H + D, s, nullptr, dPIN, H + D);
  else if ((H + D) % 4 == 0)
    hipLaunchKernelGGL(k_tr_rank1_add, dim3(2048), dim3(256), 0, s, dPIN, (long)(H + D), c->dST.as<float>(),
                       c->WsT.as<float>(), TB, H + D);
  else
    tr_gemm((int)TB, H + D, 1, c->dST.as<float>(), 1, c->WsT.as<float>(), H + D, dPIN, H + D, s, nullptr, dPIN, H + D);
  tr_zero_many({{dX1 + TB * LX1, sizeof(float) * (size_t)B * LX1}, {dX2 + TB * 2 * H, sizeof(float) * (size_t)B * 2 * H},
                {c->DC1.p, c->DC1.bytes}, {c->DC2.p, c->DC2.bytes}, {c->R1.p, c->R1.bytes}, {c->R2.p, c->R2.bytes},
                {c->DKEYS.p, c->DKEYS.bytes}, {c->DCUM.p, c->DCUM.bytes}, {c->dV.p, c->dV.bytes}, {c->dBA.p, c->dBA.bytes},
                {c->dKC.p, c->dKC.bytes}, {c->dBC.p, c->dBC.bytes}},
               s);
  // the attention backward as one launch of nq work-groups per row (k_tr_att_bwd_q; TT2_TR_ATTQ=0: the
  // two per-tile launches)
  static const bool att_q_env = [] {
    const char* e = std::getenv("TT2_TR_ATTQ");
    return !(e && e[0] == '0');
  }();
  const bool att_q = att_q_env && fused && A == 128 && F == 32 && KW == 31 && D % 4 == 0 && D <= 1024 && Tin <= 256;
  const int nq = std::min(4, NT);
  if (att_q)
    for (DevBuf* d : {&c->DF2, &c->DCUM2, &c->SC2, &c->DWGP}) TT2_HIP(hipMemsetAsync(d->p, 0, d->bytes, s));
  at.DWGP = c->DWGP.as<float>();
  // TT2_ATTQ_STAMP=<step>: k_tr_att_bwd_q stage stamps of that step -> TT2_ATTQ_STAMP_FILE (diagnostic)
  const char* aqs = std::getenv("TT2_ATTQ_STAMP");
  at.stamps = nullptr;
  at.stamp_t = aqs ? std::atoi(aqs) : -1;
  if (aqs && att_q) {
    if (c->tpStamps.bytes < sizeof(long long) * (size_t)B * 64) c->tpStamps.alloc(sizeof(long long) * (size_t)B * 64);
    TT2_HIP(hipMemsetAsync(c->tpStamps.p, 0, c->tpStamps.bytes, s));
    at.stamps = c->tpStamps.as<long long>();
  }
  // the whole reverse loop as one persistent launch when the forward ran persistent (same geometry)
  const bool tb_run = c->tb_on && fused && Tin <= TB_TMAX && tr_persist_fits(c, Tin, free_run, at.values16 != nullptr);
  c->tb_last = tb_run;
  if (tb_run) {
    tr_persist_backward(c, at, zm, Tin, T, NT, s);
    // the prenet columns of d X1 (off the recurrence): one product over all T·B rows (A = bf16(dG1) as the
    // launch wrote it, when it did)
    if (c->tb_dgr && c->blas_on && g_tr_prec == 2) {
      gemm_bf16_kc((int)TB, P, 4 * H, c->dG1.as<float>(), 4 * H, c->K1T.as<float>(), LX1, dX1, LX1, c->blasA, c->blasB,
                   c->blasP, s, false, nullptr, nullptr, c->tbDGR1.as<__bf16>());
      ++c->blas_calls;
    } else {
      tr_gemm((int)TB, P, 4 * H, c->dG1.as<float>(), 4 * H, c->K1T.as<float>(), LX1, dX1, LX1, s);
    }
  }
  for (int t = tb_run ? -1 : T - 1; t >= 0; --t) {
    const long s1 = (long)t * B;
    at.t = t;
    // (d align from the bf16 values copy measured 28.3 against 18.7 us per launch: hipcc waits
    // vmcnt(0) behind the bf16 loads of each row -- the fp32 rows stay)
    if (att_q) {
      const long o1 = (long)((t + 1) & 1) * B * Tin, o0 = (long)(t & 1) * B * Tin;
      float* dcum2 = c->DCUM2.as<float>();
      float* df2 = c->DF2.as<float>();
      float* pq2 = c->PQ2.as<float>();
      float* sc2 = c->SC2.as<float>();
      const long po1 = (long)((t + 1) & 1) * B * NT * A, po0 = (long)(t & 1) * B * NT * A;
      TrQ z{};
      z.nq = nq;
      z.dcum_in = dcum2 + o1; z.df_in = df2 + o1 * F; z.pq_in = pq2 + po1; z.sc_in = sc2 + ((t + 1) & 1) * B * 4;
      z.dcum_out = dcum2 + o0; z.df_out = df2 + o0 * F; z.pq_out = pq2 + po0; z.sc_out = sc2 + (t & 1) * B * 4;
      hipLaunchKernelGGL(k_tr_att_bwd_q, dim3(nq, B), dim3(TRQ_NT), 0, s, at, z);
    } else {
      if (A <= 128 && D <= 1024 && D % 4 == 0 && tr_e2)
        hipLaunchKernelGGL(k_tr_att_energy_bwd2, att_grid, dim3(TR_E2T), 0, s, at);
      else
        hipLaunchKernelGGL(k_tr_att_energy_bwd, att_grid, dim3(TR_AT), 0, s, at);
      hipLaunchKernelGGL(k_tr_att_conv_bwd, att_grid, dim3(256), 0, s, at);
    }
    if (fused) {  // the three per-step products of the LSTM backward, each fused with its consumer
      __bf16* dGh = c->dGh.as<__bf16>();
      TrFused f{};  // LSTM-2: d h2 = DQ·Wq^T + d PIN[t][:, :H] -> cell backward -> dG2
      f.Af = c->DQ.as<float>() + s1 * A; f.lda = A; f.Wt = c->tWq.as<__bf16>(); f.K = A; f.B = B; f.H = H;
      f.af_parts = 1;
      if (att_q) {  // the d query partials of this step's position ranges, summed by the consumer
        f.Af = c->PQ2.as<float>() + (long)(t & 1) * B * NT * A; f.lda = (long)NT * A; f.af_parts = nq; f.af_pstride = A;
      }
      f.t = t; f.layer = 1; f.z = z; f.zm = zm;
      f.G = c->G2.as<float>() + s1 * 4 * H; f.cn = c->CN2.as<float>() + s1 * H; f.c_prev = c->C2.as<float>() + s1 * H;
      f.dh_ext = dPIN + s1 * (H + D); f.ld_dh = H + D;
      f.dhz = dX2 + (s1 + B) * 2 * H + H; f.ld_dhz = 2 * H; f.DC = c->DC2.as<float>();
      f.dG = c->dG2.as<float>() + s1 * 4 * H; f.dGh = dGh; f.R = c->R2.as<float>(); f.ldr = 2 * H; f.off_r = H;
      hipLaunchKernelGGL(k_tr_fused<TF_BWD_H>, dim3(2 * H / 32), dim3(TLG_NT), 0, s, f);
      TrFused f1{};  // LSTM-1: [d h1 | d hz2_{t-1}] = dG2·K2^T (+ R2) -> cell backward -> dG1
      f1.Ah = dGh; f1.Wt = c->tK2.as<__bf16>(); f1.K = 4 * H; f1.B = B; f1.H = H;
      f1.t = t; f1.layer = 0; f1.z = z; f1.zm = zm;
      f1.G = c->G1.as<float>() + s1 * 4 * H; f1.cn = c->CN1.as<float>() + s1 * H; f1.c_prev = c->C1.as<float>() + s1 * H;
      f1.side = dX2 + s1 * 2 * H + H; f1.ld_side = 2 * H; f1.side_res = c->R2.as<float>(); f1.ld_side_res = 2 * H;
      f1.dhz = dX1 + (s1 + B) * LX1 + P + D; f1.ld_dhz = LX1; f1.DC = c->DC1.as<float>();
      f1.dG = c->dG1.as<float>() + s1 * 4 * H; f1.dGh = dGh + Bp * 4 * H; f1.R = c->R1.as<float>(); f1.ldr = LX1;
      f1.off_r = P + D;
      hipLaunchKernelGGL(k_tr_fused<TF_BWD_S>, dim3(2 * H / 16), dim3(TLG_NT), 0, s, f1);
      TrFused f3{};  // d X1[t] = dG1·K1^T + R1
      f3.Ah = dGh + Bp * 4 * H; f3.Wt = c->tK1.as<__bf16>(); f3.K = 4 * H; f3.B = B; f3.H = H;
      f3.N = LX1; f3.C = dX1 + s1 * LX1; f3.ldc = LX1; f3.residual = c->R1.as<float>(); f3.ldres = LX1;
      hipLaunchKernelGGL(k_tr_fused<TF_PLAIN>, dim3(2 * ((LX1 + 31) / 32)), dim3(TLG_NT), 0, s, f3);
    } else {
      // LSTM-2 backward: d h2 = DQ·Wq^T (raw split-K) + d PIN[t][:, :H], combined in the cell kernel
      const int kq = tr_gemm_raw(B, H, A, c->DQ.as<float>() + s1 * A, A, c->WqT.as<float>(), H, s, &c->hWq, A);
      TrLstmBwd b2{};
      b2.dh_ext = dPIN + s1 * (H + D); b2.ld_dh = H + D; b2.part = c->kpart.as<float>(); b2.ks = kq; b2.pN = H;
      b2.dhz = dX2 + (s1 + B) * 2 * H + H; b2.ld_dhz = 2 * H; b2.DC = c->DC2.as<float>();
      b2.G = c->G2.as<float>() + s1 * 4 * H; b2.cn = c->CN2.as<float>() + s1 * H; b2.c_prev = c->C2.as<float>() + s1 * H;
      b2.zm = zm; b2.t = t; b2.layer = 1; b2.B = B; b2.H = H; b2.z = z;
      b2.dG = c->dG2.as<float>() + s1 * 4 * H; b2.R = c->R2.as<float>(); b2.ldr = 2 * H; b2.off_r = H;
      hipLaunchKernelGGL(k_tr_lstm_bwd, dim3(bh), dim3(256), 0, s, b2);
      // dX2 = dG2·K2^T + R2 (raw split-K): columns [0,H) are d h1_new (consumed by the LSTM-1
      // backward), columns [H,2H) = d hz2_{t-1} are written to dX2[t] by the same kernel
      const int kx = tr_gemm_raw(B, 2 * H, 4 * H, c->dG2.as<float>() + s1 * 4 * H, 4 * H, c->K2T.as<float>(), 2 * H, s,
                                 &c->hK2, 4 * H);
      TrLstmBwd b1{};
      b1.dh_ext = nullptr; b1.ld_dh = 0; b1.part = c->kpart.as<float>(); b1.ks = kx; b1.pN = 2 * H;
      b1.side = dX2 + s1 * 2 * H + H; b1.ld_side = 2 * H; b1.side_res = c->R2.as<float>(); b1.ld_side_res = 2 * H;
      b1.dhz = dX1 + (s1 + B) * LX1 + P + D; b1.ld_dhz = LX1; b1.DC = c->DC1.as<float>();
      b1.G = c->G1.as<float>() + s1 * 4 * H; b1.cn = c->CN1.as<float>() + s1 * H; b1.c_prev = c->C1.as<float>() + s1 * H;
      b1.zm = zm; b1.t = t; b1.layer = 0; b1.B = B; b1.H = H; b1.z = z;
      b1.dG = c->dG1.as<float>() + s1 * 4 * H; b1.R = c->R1.as<float>(); b1.ldr = LX1; b1.off_r = P + D;
      hipLaunchKernelGGL(k_tr_lstm_bwd, dim3(bh), dim3(256), 0, s, b1);
      tr_gemm(B, LX1, 4 * H, c->dG1.as<float>() + s1 * 4 * H, 4 * H, c->K1T.as<float>(), LX1, dX1 + s1 * LX1, LX1, s,
              nullptr, c->R1.as<float>(), LX1, ACT_NONE, &c->hK1, 4 * H);
    }
    if (free_run && t > 0 && !c->feed[t]) {
      // step t consumed frame t-1: d prenet input -> d frame t-1 (dFR, for the projection weight
      // gradients after the loop) and through the frame projection into d [h2 | ctx] of step t-1
      // (dPIN, consumed by the next iteration)
      float* dz = c->sDZ.as<float>();
      float* dp = c->sDP.as<float>();
      float* dx = c->sDX.as<float>();
      hipLaunchKernelGGL(k_tr_prenet_bwd, dim3(nblk((long)B * P)), dim3(256), 0, s, dX1 + s1 * LX1, (long)LX1,
                         X1 + s1 * LX1, (long)LX1, (long)B, P, dz);
      tr_gemm(B, P, P, dz, P, c->Wp2T.as<float>(), P, dp, P, s);
      hipLaunchKernelGGL(k_tr_prenet_bwd, dim3(nblk((long)B * P)), dim3(256), 0, s, dp, (long)P,
                         c->P1.as<float>() + s1 * P, (long)P, (long)B, P, dz);
      tr_gemm(B, NM, P, dz, P, c->W1T.as<float>(), NM, dx, NM, s);
      float* dfr = c->dFR.as<float>() + (s1 - B) * NR + (R - 1) * NM;  // the last of step t-1's r frames
      tr_gemm(B, NM, P, dz, P, c->W1T.as<float>(), NM, dfr, NR, s, nullptr, dfr, NR);
      float* dpin = dPIN + (s1 - B) * (H + D);
      tr_gemm(B, H + D, NM, dx, NM, c->WfT.as<float>() + (long)(R - 1) * NM * (H + D), H + D, dpin, H + D, s, nullptr,
              dpin, H + D);
    }
  }

  if (att_q && !tb_run)  // d query of step 0 (the later steps' sums were written by the launch after them)
    hipLaunchKernelGGL(k_tr_dq_sum, dim3(B), dim3(128), 0, s, c->PQ2.as<float>(), NT, nq, A, c->DQ.as<float>());
  if (at.stamps) {
    std::vector<long long> h((size_t)B * 64);
    TT2_HIP(hipMemcpyAsync(h.data(), at.stamps, h.size() * sizeof(long long), hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
    const char* fn = std::getenv("TT2_ATTQ_STAMP_FILE");
    if (FILE* f = std::fopen(fn ? fn : "attq_stamps.bin", "wb")) {
      std::fwrite(h.data(), sizeof(long long), h.size(), f);
      std::fclose(f);
    }
    at.stamps = nullptr;
  }
  // ---- weight gradients over all T·B rows ----
  float* TBUF = c->TBUF.as<float>();
  const int TBi = (int)TB;
  const bool dgt = tb_run && c->tb_dgt;
  tr_gemm_xtg(LX1, 4 * H, TBi, X1, LX1, c->dG1.as<float>(), 4 * H, gvar(c, L1V("kernel")), 4 * H, TBUF, s,
              dgt ? c->tbDGT1.as<__bf16>() : nullptr);
  tr_colsum(c, c->dG1.as<float>(), TB, 4 * H, 4 * H, gvar(c, L1V("bias")), s);
  tr_gemm_xtg(2 * H, 4 * H, TBi, X2, 2 * H, c->dG2.as<float>(), 4 * H, gvar(c, L2V("kernel")), 4 * H, TBUF, s,
              dgt ? c->tbDGT2.as<__bf16>() : nullptr);
  tr_colsum(c, c->dG2.as<float>(), TB, 4 * H, 4 * H, gvar(c, L2V("bias")), s);
  tr_transpose(PIN, TB, H + D, H + D, TBUF, TB, s);
  tr_gemm(H, A, TBi, TBUF, TB, c->DQ.as<float>(), A, gvar(c, vn("decoder/query_layer/kernel")), A, s);
  tr_gemm(H + D, NR, TBi, TBUF, TB, c->dFR.as<float>(), NR, gvar(c, FPV("kernel")), NR, s);
  tr_gemm(H + D, R, TBi, TBUF, TB, c->dST.as<float>(), R, gvar(c, SPV("kernel")), R, s);
  tr_colsum(c, c->dFR.as<float>(), TB, NR, NR, gvar(c, FPV("bias")), s);
  tr_colsum(c, c->dST.as<float>(), TB, R, R, gvar(c, SPV("bias")), s);
  // prenet
  hipLaunchKernelGGL(k_tr_prenet_bwd, dim3(nblk(TB * P)), dim3(256), 0, s, dX1, (long)LX1, X1, (long)LX1, TB, P,
                     c->dZ.as<float>());
  tr_transpose(c->P1.as<float>(), TB, P, P, TBUF, TB, s);
  tr_gemm(P, P, TBi, TBUF, TB, c->dZ.as<float>(), P, gvar(c, PRV(2, "kernel")), P, s);
  tr_colsum(c, c->dZ.as<float>(), TB, P, P, gvar(c, PRV(2, "bias")), s);
  tr_gemm(TBi, P, P, c->dZ.as<float>(), P, c->Wp2T.as<float>(), P, c->dPre.as<float>(), P, s);
  hipLaunchKernelGGL(k_tr_prenet_bwd, dim3(nblk(TB * P)), dim3(256), 0, s, c->dPre.as<float>(), (long)P,
                     c->P1.as<float>(), (long)P, TB, P, c->dZ.as<float>());
  tr_transpose(c->XIN.as<float>(), TB, NM, NM, TBUF, TB, s);
  tr_gemm(NM, P, TBi, TBUF, TB, c->dZ.as<float>(), P, gvar(c, PRV(1, "kernel")), P, s);
  tr_colsum(c, c->dZ.as<float>(), TB, P, P, gvar(c, PRV(1, "bias")), s);
  // attention parameters: sums of the per-row partials
  const long BNT = (long)B * NT;
  tr_colsum(c, c->dV.as<float>(), BNT, A, A, gvar(c, LAV("attention_variable_projection")), s);
  tr_colsum(c, c->dBA.as<float>(), BNT, A, A, gvar(c, LAV("attention_bias")), s);
  {  // d W_loc = Σ_{t,b,j} f ⊗ du over all T·B·Tin rows
    const long R = TB * Tin;
    // one streaming fp32-MFMA pass (k_tr_dwloc), partials [nbk][F·A] in TBUF: at most 512 blocks
    // and never more than TBUF holds (small T·B configurations have a small TBUF)
    const long cap = (long)(c->TBUF.bytes / sizeof(float)) / ((long)F * A);
    const long cap32 = (long)(c->TBUF.bytes / sizeof(float)) / (32L * A);
    if (att_q || tb_run) {  // G per (row, range) slot (k_tr_att_bwd_q / the persistent backward); row 31 = Σ du = d b_a
      tr_colsum(c, c->DWGP.as<float>(), BNT, 32 * A, 32L * A, c->DWG.as<float>(), s);
      TT2_HIP(hipMemcpyAsync(c->DWG.as<float>() + 31L * A, gvar(c, LAV("attention_bias")), sizeof(float) * (size_t)A,
                             hipMemcpyDeviceToDevice, s));
      hipLaunchKernelGGL(k_tr_dwloc_fin, dim3((F * A + 255) / 256), dim3(256), 0, s, c->DWG.as<float>(),
                         pvar(c, LAV("location_features_convolution/kernel")),
                         pvar(c, LAV("location_features_convolution/bias")), F, A, KW,
                         gvar(c, LAV("location_features_layer/kernel")));
    } else if (tr_dwloc_cum_ok(c) && cap32 >= 1) {
      const long nb = std::min<long>(512, cap32);
      const long rpb = ((R + nb - 1) / nb + 31) / 32 * 32;
      const int nbk = (int)((R + rpb - 1) / rpb);
      hipLaunchKernelGGL(k_tr_dwloc_cum, dim3(nbk), dim3(256), 0, s, c->CUM.as<float>(), c->TH.as<float>(), R, Tin, A, KW,
                         rpb, TBUF);
      tr_colsum(c, TBUF, nbk, 32 * A, 32L * A, c->DWG.as<float>(), s);
      hipLaunchKernelGGL(k_tr_dwloc_fin, dim3((F * A + 255) / 256), dim3(256), 0, s, c->DWG.as<float>(),
                         pvar(c, LAV("location_features_convolution/kernel")),
                         pvar(c, LAV("location_features_convolution/bias")), F, A, KW,
                         gvar(c, LAV("location_features_layer/kernel")));
    } else if (F <= 32 && A <= 128 && cap >= 1) {
      const long nb = std::min<long>(512, cap);
      const long rpb = ((R + nb - 1) / nb + 31) / 32 * 32;
      const int nbk = (int)((R + rpb - 1) / rpb);
      TT2_CHECK((long)nbk * F * A * (long)sizeof(float) <= (long)c->TBUF.bytes, TT2_ERR_STATE,
                "d W_loc partials exceed TBUF");
      hipLaunchKernelGGL(k_tr_dwloc, dim3(nbk), dim3(256), 0, s, c->FALL.as<float>(), c->TH.as<float>(), R, F, A, rpb,
                         TBUF);
      tr_colsum(c, TBUF, nbk, F * A, (long)F * A, gvar(c, LAV("location_features_layer/kernel")), s);
    } else {
      tr_transpose(c->FALL.as<float>(), R, F, F, TBUF, R, s);
      tr_gemm(F, A, (int)R, TBUF, R, c->TH.as<float>(), A, gvar(c, LAV("location_features_layer/kernel")), A, s);
    }
  }
  if (tb_run) {  // d Kc, d bc from the summed G (train_bwd_persist.h)
    tb_loc_grads(c->DWG.as<float>(), pvar(c, LAV("location_features_layer/kernel")), F, A, KW,
                 gvar(c, LAV("location_features_convolution/kernel")), gvar(c, LAV("location_features_convolution/bias")),
                 s);
  } else {
    tr_colsum(c, c->dKC.as<float>(), BNT, KW * F, (long)KW * F,
              gvar(c, LAV("location_features_convolution/kernel")), s);
    tr_colsum(c, c->dBC.as<float>(), BNT, F, F, gvar(c, LAV("location_features_convolution/bias")), s);
  }
  // memory: d values = Σ_t align_t^T · dctx_t (+ keys path), memory_layer kernel
  // (one launch for all rows: the per-row GEMMs were 64 launches + split-K combines, 1.37 ms at configs[4])
  hipLaunchKernelGGL(k_tr_dval, dim3((D + 127) / 128, (Tin + DV_JT - 1) / DV_JT, B), dim3(512), 0, s, c->ALIGN.as<float>(),
                     c->DCTX.as<float>(), B, Tin, T, D, c->DVAL.as<float>());
  TT2_HIP(hipGetLastError());
  tr_transpose(c->values.as<float>(), (long)B * Tin, D, D, TBUF, (long)B * Tin, s);
  tr_gemm(D, A, B * Tin, TBUF, (long)B * Tin, c->DKEYS.as<float>(), A, gvar(c, vn("memory_layer/kernel")), A, s);
  tr_gemm(B * Tin, D, A, c->DKEYS.as<float>(), A, c->WmT.as<float>(), D, c->DVAL.as<float>(), D, s, nullptr,
          c->DVAL.as<float>(), D);
  hipLaunchKernelGGL(k_tr_mask_rows, dim3(nblk((long)B * Tin * D)), dim3(256), 0, s, c->DVAL.as<float>(), lens, B, Tin,
                     D, c->DMEM.as<float>());
  g_tr_kpart = nullptr;
  g_tr_prec = 0;
  g_tr_ctx = nullptr;
}

// L2 regularisation of the regularised kernels (after every gradient of the step has landed)
static void tr_regularize(tt2_train_ctx* c, hipStream_t s) {
  if (!c->reg_segs.p) {  // the regularised variables' (offset, size), fixed at create
    std::vector<long2> seg;
    for (const auto& v : c->vars)
      if (v.reg) seg.push_back(make_long2((long)v.off, (long)v.n));
    c->nreg = (int)seg.size();
    c->reg_segs.alloc(sizeof(long2) * std::max<size_t>(seg.size(), 1));
    if (!seg.empty()) TT2_HIP(hipMemcpy(c->reg_segs.p, seg.data(), sizeof(long2) * seg.size(), hipMemcpyHostToDevice));
  }
  if (c->nreg)
    hipLaunchKernelGGL(k_tr_reg, dim3(64, c->nreg), dim3(256), 0, s, c->params.as<float>(), c->grads,
                       c->reg_segs.as<long2>(), c->cfg.reg_weight, c->part.as<float>());
  hipLaunchKernelGGL(k_tr_sum_final, dim3(1), dim3(256), 0, s, c->part.as<float>(), 64 * c->nreg, c->cfg.reg_weight,
                     c->red.as<float>() + 2, 0);
}

// ---- front end (cfg.frontend): encoder, reference encoders, GST in training mode -------------------
// The step starts from ids / reference mels: forward builds the memory the decoder slice consumes
// (tacotron.py:215-308), backward continues from the decoder's d memory (DMEM) into every front-end
// variable (train_front.hip kernels + gemm.hip products).
static std::string fe_conv_scope(int i) {
  return vn("encoder_convolutions/conv_layer_") + std::to_string(i) + "_encoder_convolutions/";
}
static std::string fe_ref_scope(const tt2_train_ctx* c, int r) {
  return vn(c->f_adain ? "refnet/" : r == 0 ? "refnet_emt/" : "refnet_spk/");
}
// conv layer scope of stack r in conv2d_i/: AdaIN's two stacks share 'refnet/conv2d_i' and
// tf.layers uniquifies the second (emotion) layer's default name (modules.py:84-87)
static std::string fe_ref_conv(const tt2_train_ctx* c, int r) { return c->f_adain && r == 0 ? "conv2d_1/" : "conv2d/"; }
// stride of refnet layer i: (2, 2) everywhere, AdaIN (2,2),(2,2),(1,1)x4 (tacotron.py:237)
static int fe_ref_stride(const tt2_train_ctx* c, int i) { return c->f_adain && i >= 2 ? 1 : 2; }
static std::string fe_mh_scope(int r) { return vn(r == 0 ? "Multihead-attention-emt/" : "Multihead-attention-spk/"); }
static std::string fe_lstm_scope(int d) {
  return vn(d == 0 ? "encoder_LSTM/bidirectional_rnn/fw/lstm_cell/" : "encoder_LSTM/bidirectional_rnn/bw/lstm_cell/");
}
static bool fe_regularized(const std::string& n) {  // tacotron.py:865-867 (oracle/train_ref.py regularized)
  return !(n.find("bias") != std::string::npos || n.find("Bias") != std::string::npos ||
           n.find("_projection") != std::string::npos || n.find("inputs_embedding") != std::string::npos ||
           n.find("RNN") != std::string::npos || n.find("LSTM") != std::string::npos);
}

static void tr_front_build_vars(tt2_train_ctx* c, const std::function<void(const std::string&, std::vector<int64_t>, bool)>& add) {
  const auto& f = c->cfg;
  const int E = f.embedding_dim, C = f.enc_conv_channels, K = f.enc_conv_kernel, U = f.encoder_lstm_units;
  auto addr = [&](const std::string& n, std::vector<int64_t> sh) { add(n, sh, fe_regularized(n)); };
  addr(vn("inputs_embedding"), {f.n_symbols, E});
  for (int i = 1; i <= f.enc_conv_layers; ++i) {
    const std::string s = fe_conv_scope(i);
    addr(s + "conv1d/kernel", {K, i == 1 ? E : C, C});
    addr(s + "conv1d/bias", {C});
    addr(s + "batch_normalization/gamma", {C});
    addr(s + "batch_normalization/beta", {C});
    add(s + "batch_normalization/moving_mean", {C}, false);
    add(s + "batch_normalization/moving_variance", {C}, false);
  }
  for (int d = 0; d < 2; ++d) {
    addr(fe_lstm_scope(d) + "kernel", {C + U, 4 * U});
    addr(fe_lstm_scope(d) + "bias", {4 * U});
  }
  const int RD = f.reference_depth, tokd = f.style_embed_depth / f.num_heads, A = f.style_att_dim, dh = A / f.num_heads;
  if (c->f_adain) {  // 'refnet' (modules.py:66-107): both conv stacks per layer, then GRU + dense
    const std::string rs = fe_ref_scope(c, 1);
    int ci = 1;
    for (int i = 0; i < 6; ++i) {
      const std::string s = rs + "conv2d_" + std::to_string(i) + "/";
      for (int r = 1; r >= 0; --r) {  // speaker stack first (conv2d/), then emotion (conv2d_1/)
        addr(s + fe_ref_conv(c, r) + "kernel", {3, 3, ci, f.reference_filters[i]});
        addr(s + fe_ref_conv(c, r) + "bias", {f.reference_filters[i]});
      }
      ci = f.reference_filters[i];
    }
    addr(rs + "rnn/gru_cell/gates/kernel", {c->f_gin + RD, 2 * RD});
    addr(rs + "rnn/gru_cell/gates/bias", {2 * RD});
    addr(rs + "rnn/gru_cell/candidate/kernel", {c->f_gin + RD, RD});
    addr(rs + "rnn/gru_cell/candidate/bias", {RD});
    addr(rs + "dense/kernel", {RD, 128});
    addr(rs + "dense/bias", {128});
    return;
  }
  for (int r = 0; r < c->f_nref; ++r) {
    const std::string rs = fe_ref_scope(c, r);
    int ci = 1;
    for (int i = 0; i < 6; ++i) {
      const std::string s = rs + "conv2d_" + std::to_string(i) + "/";
      addr(s + "conv2d/kernel", {3, 3, ci, f.reference_filters[i]});
      addr(s + "conv2d/bias", {f.reference_filters[i]});
      addr(s + "batch_normalization/gamma", {f.reference_filters[i]});
      addr(s + "batch_normalization/beta", {f.reference_filters[i]});
      add(s + "batch_normalization/moving_mean", {f.reference_filters[i]}, false);
      add(s + "batch_normalization/moving_variance", {f.reference_filters[i]}, false);
      ci = f.reference_filters[i];
    }
    addr(rs + "rnn/gru_cell/gates/kernel", {c->f_gin + RD, 2 * RD});
    addr(rs + "rnn/gru_cell/gates/bias", {2 * RD});
    addr(rs + "rnn/gru_cell/candidate/kernel", {c->f_gin + RD, RD});
    addr(rs + "rnn/gru_cell/candidate/bias", {RD});
    addr(rs + "dense/kernel", {RD, 128});
    addr(rs + "dense/bias", {128});
    if (!f.use_gst) continue;  // hp.use_gst = False: no style tokens / style attention (tacotron.py:284-291)
    addr(vn(r == 0 ? "style_tokens_emt" : "style_tokens_spk"), {f.num_gst, tokd});
    const std::string m = fe_mh_scope(r);
    addr(m + "conv1d/kernel", {1, 128, A});
    addr(m + "conv1d/bias", {A});
    addr(m + "conv1d_1/kernel", {1, tokd, A});
    addr(m + "conv1d_1/bias", {A});
    addr(m + "attention_v", {dh});
    addr(m + "attention_g", {});
    addr(m + "attention_b", {dh});
  }
  // Style_Emb_Disc dense layers (modules.py:626-644, tacotron.py:489-493; oracle style_disc_var_names)
  for (int r = 0; r < c->f_nref; ++r) {
    const int n = r == 0 ? f.n_emt : f.n_spk;
    if (n <= 0) continue;
    const std::string sd = vn(r == 0 ? "style_disc_emt/dense/" : "style_disc_spk/dense/");
    addr(sd + "kernel", {128, n});
    addr(sd + "bias", {n});
  }
}

// the encoder BiLSTM steps as fused products (k_tr_fused TF_EFWD / TF_EBWD): bf16 step, B <= 64,
// U a multiple of 128; TT2_TR_FUSED=0 keeps the split products + cell launches
static bool fe_enc_fused(tt2_train_ctx* c) {
  const char* fe = std::getenv("TT2_TR_FUSED");
  const int U = c->cfg.encoder_lstm_units;
  return !(fe && fe[0] == '0') && g_tr_prec == 2 && c->B <= 64 && U % 128 == 0;
}

static void tr_front_alloc(tt2_train_ctx* c) {
  const auto& f = c->cfg;
  const long B = c->B, T = c->Tin, C = f.enc_conv_channels, E = f.embedding_dim, U = f.encoder_lstm_units;
  const long BT = B * T, K = f.enc_conv_kernel;
  auto a = [](DevBuf& d, long n) { d.alloc(sizeof(float) * (size_t)std::max<long>(n, 1)); };
  a(c->fEX, BT * E);
  const char* pe = std::getenv("TT2_PN_PLANES");  // 0: implicit-im2col gemm_x3_kernel convs here too
  // one plane buffer serves the embedding (stride E) and the conv layers (stride C): the pad rows
  // are zeroed once per shape, so the two strides must agree or the stride-E frames land on the
  // stride-C pad rows (the im2col path serves E != C)
  if ((!pe || std::atoi(pe) != 0) && c->cfg.precision && C % 64 == 0 && E == C && (K & 1) &&
      K <= 2 * CX_P + 1) {
    const long W = std::max(C, E), Wr = (W + 255) / 256 * 256;
    c->fePl.alloc((size_t)cx_rows((int)B, (int)T) * W * 2);
    c->feWt.alloc((size_t)Wr * K * W * 2);
  }
  for (int i = 0; i < f.enc_conv_layers; ++i) {
    a(c->fEA[i], BT * C);
    a(c->fEY[i + 1], BT * C);
  }
  a(c->fXP, BT * 8 * U); a(c->fGZ, 2 * B * 4 * U); a(c->fGA, 2 * T * B * 4 * U); a(c->fCN, 2 * T * B * U);
  a(c->fCS, 2 * (T + 1) * B * U); a(c->fHS, 2 * (T + 1) * B * U); a(c->fENC, BT * 2 * U);
  a(c->fMEM, BT * c->D); a(c->fSTY, B * (c->D - 2 * U)); a(c->fDSTY, B * (c->D - 2 * U));
  a(c->fDZ, 2 * T * B * 4 * U); a(c->fDHC, 2 * B * U); a(c->fDCC, 2 * B * U); a(c->fDHP, 2 * B * U);
  a(c->fdXP, BT * 8 * U); a(c->fdA, BT * std::max(C, E)); a(c->fdB, BT * std::max(C, E));
  a(c->fLWxT, 2 * 4 * U * C); a(c->fLWhT, 2 * 4 * U * U);
  {  // bf16 TF-layout operands of the fused encoder LSTM steps (k_tr_fused TF_EFWD / TF_EBWD)
    const long Bp = (B + 31) & ~31L;
    auto h = [](DevBuf& d, long n) { d.alloc(2 * (size_t)std::max<long>(n, 1)); };
    h(c->fTWf, 2 * 4 * U * U); h(c->fTWb, 2 * 4 * U * U); h(c->fHSh, 2 * (T + 1) * Bp * U); h(c->fDZh, 2 * 2 * Bp * 4 * U);
  }
  // reference encoders at max_T_ref
  const int RD = f.reference_depth, nm = c->NM;
  long fbuf = BT * K * std::max(C, E);  // encoder im2col^T
  // fDY / fDZc hold the refnet conv activations' gradients AND the encoder convs' BN backward
  // (dy, dz: B·T_in·C each)
  long mmax = BT * C;
  long wt_conv2d = 1;  // largest 3x3 conv2d kernel transpose [fo][9·ci]
  int H = f.max_T_ref, W = nm, ci = 1;
  for (int i = 0; i < 6; ++i) {
    const int st = fe_ref_stride(c, i), Ho = (H + st - 1) / st, Wo = (W + st - 1) / st, fo = f.reference_filters[i];
    const long M = B * Ho * Wo;
    for (int r = 0; r < c->f_nref; ++r) {
      a(c->fRA[r][i], c->f_adain ? 1 : M * fo);  // pre-BN activations (AdaIN: no batch norm)
      a(c->fRY[r][i], M * fo);
    }
    fbuf = std::max(fbuf, 9L * ci * M);
    mmax = std::max(mmax, std::max(M * fo, B * (long)H * W * ci));
    wt_conv2d = std::max(wt_conv2d, 9L * ci * fo);
    H = Ho; W = Wo; ci = fo;
  }
  const long T2 = H;
  c->f_T2max = (int)T2;
  // FB also holds the transposes of the GRU states / inputs over all T2·B rows and the BiLSTM states
  fbuf = std::max({fbuf, T2 * B * std::max<long>((long)W * ci, RD), BT * U, BT * C});
  for (int r = 0; r < c->f_nref; ++r) {
    a(c->fXG[r], B * T2 * 3 * RD); a(c->fGR[r], T2 * B * RD); a(c->fGU[r], T2 * B * RD); a(c->fGCC[r], T2 * B * RD);
    a(c->fGRH[r], T2 * B * RD); a(c->fHG[r], (T2 + 1) * B * RD); a(c->fREF[r], B * 128);
  }
  a(c->fGG, B * 2 * RD); a(c->fGC, B * RD);
  if (c->f_adain) {
    const long nmap = T2 * B * (long)W * ci;
    a(c->fADX, nmap); a(c->fDYE, std::max(mmax, nmap));
    a(c->fADM, 2L * B * ci * 2); a(c->fADS, (long)B * ci * 2);
    mmax = std::max(mmax, nmap);
  }
  a(c->fFBUF, fbuf); a(c->fDY, mmax); a(c->fDY2, mmax); a(c->fDZc, mmax);
  // the direct conv2d kernel gradient sums its partial rows with tr_colsum over 9·ci·fo columns
  if (c->part.bytes < sizeof(float) * (size_t)(wt_conv2d + 4096)) c->part.alloc(sizeof(float) * (size_t)(wt_conv2d + 4096));
  const int ntok = f.num_gst, tokd = f.style_embed_depth / f.num_heads, A = f.style_att_dim, dh = A / f.num_heads;
  a(c->fGq, B * A); a(c->fGkk, B * ntok * A); a(c->fGv, B * ntok * tokd); a(c->fGnv, B * dh); a(c->fGbb, B * dh);
  a(c->fGsum, ntok * A + ntok * tokd + 2 * dh);
  a(c->sXREF, 2 * B * 128); a(c->sDL, B * std::max(1, std::max(f.n_emt, f.n_spk))); a(c->sOM, B * B);
  c->sLAB.alloc(sizeof(int) * (size_t)(2 * B));
  a(c->fdREF, B * 128); a(c->fDZD, B * 128); a(c->fDH, B * RD); a(c->fDHA, B * RD); a(c->fDRH, B * RD);
  a(c->fDCP, T2 * B * RD); a(c->fDGP, T2 * B * 2 * RD); a(c->fDXG, B * T2 * 3 * RD);
  // transposed / flipped weight scratch: refnet conv2d kernels, GRU gates + candidate, dense, GST
  // query, and the encoder conv flip K·cin·C with cin = E for the first layer
  a(c->fWT, std::max<long>({wt_conv2d, 3L * RD * std::max<long>(c->f_gin, RD), 128L * RD, 128L * A,
                            (long)K * std::max(C, E) * C}));
  a(c->fBN, 2L * (f.enc_conv_layers + 6 * c->f_nref) * 512);
  a(c->fpart, 64L * 2 * 512 + 1024);
}

// batch statistics over M rows of [M][C] into mean / var (k_pn_colstat: biased variance)
static void fe_stats(tt2_train_ctx* c, const float* x, long M, int C, float* mean, float* var, hipStream_t s) {
  const int S = tr_splits(M, C, 64L * 512);
  const unsigned CT = (unsigned)((C + tr_tw(C) - 1) / tr_tw(C));
  float* part = c->fpart.as<float>();
  hipLaunchKernelGGL(k_pn_colstat_part, dim3(CT, S), dim3(256), 0, s, x, M, C, nullptr, 0, part);
  hipLaunchKernelGGL(k_pn_colstat_final, dim3((C + 31) / 32), dim3(TR_FIN), 0, s, part, S, C, 1.0f / (float)M, mean);
  hipLaunchKernelGGL(k_pn_colstat_part, dim3(CT, S), dim3(256), 0, s, x, M, C, mean, 1, part);
  hipLaunchKernelGGL(k_pn_colstat_final, dim3((C + 31) / 32), dim3(TR_FIN), 0, s, part, S, C, 1.0f / (float)M, var);
}
// BN backward (batch statistics) from dy -> dz (act: 0 none, 2 relu' from the pre-BN activation)
static void fe_bn_bwd(tt2_train_ctx* c, const float* dxn, const uint8_t* keep, const float* a, long M, int C,
                      const float* mean, const float* var, const std::string& sc, int act, float* dy, float* dz,
                      hipStream_t s, __bf16* planes = nullptr, int T = 1) {
  const int S = tr_splits(M, C, 64L * 512);
  float* part = c->fpart.as<float>();
  float* sums = part + 64L * 2 * 512;
  const float eps = c->cfg.bn_eps;
  hipLaunchKernelGGL(k_pn_bn_bwd_part, dim3((unsigned)((C + tr_tw(C) - 1) / tr_tw(C)), S), dim3(256), 0, s, dxn, keep,
                     a, M, C, mean, var, eps, dy, part);
  hipLaunchKernelGGL(k_pn_bn_bwd_final, dim3((C + 31) / 32), dim3(TR_FIN), 0, s, part, S, C, sums,
                     gvar(c, sc + "batch_normalization/gamma"), gvar(c, sc + "batch_normalization/beta"));
  hipLaunchKernelGGL(k_pn_bn_bwd_dz, dim3(nblk(M * C)), dim3(256), 0, s, dy, a, M, C, mean, var, eps,
                     pvar(c, sc + "batch_normalization/gamma"), sums, act, dz, planes, T);
}

// fp32 rows [B·T][C] (batch-major) -> the padded bf16 planes of conv_bf16_planes (frame rows only)
__global__ void k_rows_to_planes(const float* __restrict__ x, long M, int C, int T, __bf16* __restrict__ planes) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M * C) pn_plane_put(planes, T, i, C, x[i]);
}

static FeGst fe_gst_args(tt2_train_ctx* c, int r, int B) {
  const auto& f = c->cfg;
  const std::string m = fe_mh_scope(r);
  FeGst g{};
  g.ref = c->fREF[r].as<float>();
  g.tokens = pvar(c, vn(r == 0 ? "style_tokens_emt" : "style_tokens_spk"));
  g.wq = pvar(c, m + "conv1d/kernel"); g.bq = pvar(c, m + "conv1d/bias");
  g.wk = pvar(c, m + "conv1d_1/kernel"); g.bk = pvar(c, m + "conv1d_1/bias");
  g.v = pvar(c, m + "attention_v"); g.g = pvar(c, m + "attention_g"); g.bb = pvar(c, m + "attention_b");
  g.N = B; g.ntok = f.num_gst; g.tokd = f.style_embed_depth / f.num_heads; g.A = f.style_att_dim; g.heads = f.num_heads;
  g.refd = 128;
  g.style = c->fSTY.as<float>(); g.style_ld = c->D - 2 * f.encoder_lstm_units; g.style_off = r * f.style_embed_depth;
  g.dstyle = c->fDSTY.as<float>();
  g.dq = c->fGq.as<float>(); g.pdkk = c->fGkk.as<float>(); g.pdv = c->fGv.as<float>(); g.pdnv = c->fGnv.as<float>();
  g.pdbb = c->fGbb.as<float>();
  return g;
}

static void tr_front_forward(tt2_train_ctx* c, const int* ids, const int* lens, const float* const* refs, int T_ref,
                             const uint8_t* encm, const uint8_t* enczm, int T, hipStream_t s) {
  const auto& f = c->cfg;
  const int B = c->B, E = f.embedding_dim, C = f.enc_conv_channels, K = f.enc_conv_kernel, U = f.encoder_lstm_units;
  const long M = (long)B * T;
  const float eps = f.bn_eps;
  float* BN = c->fBN.as<float>();
  fe_embed(ids, pvar(c, vn("inputs_embedding")), M, E, c->fEX.as<float>(), s);
  // EncoderConvolutions (modules.py:251-280, conv1d() :485-497 with bnorm 'after'): conv -> ReLU ->
  // BN (batch statistics over all B·T positions) -> dropout(0.5, keep bits)
  // bf16 conv over padded planes (conv_bf16_planes, as the Postnet's): planes of the embedding here,
  // of each layer's output from its BN forward; pad rows zeroed once per shape
  const bool planes = c->fePl.p && g_tr_prec == 2;
  __bf16* pl = reinterpret_cast<__bf16*>(c->fePl.p);
  __bf16* wt = reinterpret_cast<__bf16*>(c->feWt.p);
  if (planes) {
    if (c->fe_pl_B != B || c->fe_pl_T != T) {
      TT2_HIP(hipMemsetAsync(c->fePl.p, 0, c->fePl.bytes, s));
      c->fe_pl_B = B;
      c->fe_pl_T = T;
    }
    hipLaunchKernelGGL(k_rows_to_planes, dim3(nblk(M * E)), dim3(256), 0, s, c->fEX.as<float>(), M, E, T, pl);
  }
  for (int i = 0; i < f.enc_conv_layers; ++i) {
    const std::string sc = fe_conv_scope(i + 1);
    const int cin = i == 0 ? E : C;
    if (planes) {
      kc_transpose_bf16(pvar(c, sc + "conv1d/kernel"), K * cin, C, C, wt, K * cin, (C + 255) / 256 * 256, s);
      conv_bf16_planes(pl, cin, B, T, K, wt, (long)K * cin, C, pvar(c, sc + "conv1d/bias"), ACT_RELU,
                       c->fEA[i].as<float>(), C, s);
    } else {
      GemmArgs g;
      g.a_mode = A_CONV1D; g.M = (int)M; g.N = C; g.T = T; g.kw = K; g.pad = (K - 1) / 2; g.C = cin;
      g.A = i == 0 ? c->fEX.as<float>() : c->fEY[i].as<float>(); g.xs_b = (long)T * cin; g.xs_t = cin; g.K = K * cin;
      g.Bw = pvar(c, sc + "conv1d/kernel"); g.ldb = C; g.Cout = c->fEA[i].as<float>(); g.ldc = C;
      g.bias = pvar(c, sc + "conv1d/bias"); g.act = ACT_RELU;
      tr_gemm_run(g, s);
    }
    float* mean = BN + (long)i * 2 * 512;
    float* var = mean + 512;
    fe_stats(c, c->fEA[i].as<float>(), M, C, mean, var, s);
    hipLaunchKernelGGL(k_pn_bn_fwd, dim3(nblk(M * C)), dim3(256), 0, s, c->fEA[i].as<float>(), M, C, mean, var,
                       pvar(c, sc + "batch_normalization/gamma"), pvar(c, sc + "batch_normalization/beta"), eps,
                       encm ? encm + (long)i * M * C : nullptr, c->fEY[i + 1].as<float>(),
                       planes && i + 1 < f.enc_conv_layers ? pl : nullptr, T);
  }
  // EncoderRNN (modules.py:283-323): input projections of both directions for every position
  const float* X = c->fEY[f.enc_conv_layers].as<float>();
  for (int d = 0; d < 2; ++d)
    tr_gemm((int)M, 4 * U, C, X, C, pvar(c, fe_lstm_scope(d) + "kernel"), 4 * U, c->fXP.as<float>() + d * 4 * U, 8 * U,
            s, pvar(c, fe_lstm_scope(d) + "bias"));
  TT2_HIP(hipMemsetAsync(c->fENC.p, 0, sizeof(float) * (size_t)M * 2 * U, s));
  for (int d = 0; d < 2; ++d) {  // zero initial states
    TT2_HIP(hipMemsetAsync(c->fCS.as<float>() + (long)d * (T + 1) * B * U, 0, sizeof(float) * (size_t)B * U, s));
    TT2_HIP(hipMemsetAsync(c->fHS.as<float>() + (long)d * (T + 1) * B * U, 0, sizeof(float) * (size_t)B * U, s));
  }
  FeLstm l{};
  l.XP = c->fXP.as<float>(); l.GZ = c->fGZ.as<float>(); l.GA = c->fGA.as<float>(); l.CN = c->fCN.as<float>();
  l.CS = c->fCS.as<float>(); l.HS = c->fHS.as<float>(); l.ENC = c->fENC.as<float>(); l.zm = enczm; l.lens = lens;
  l.B = B; l.T = T; l.U = U; l.zo = f.zoneout;
  if (fe_enc_fused(c)) {  // both directions' recurrent product + cell in one launch per step
    const long Bp = (B + 31) & ~31L;
    for (int d = 0; d < 2; ++d)
      hipLaunchKernelGGL(k_tr_tf_weights_f32, dim3(1024), dim3(256), 0, s, pvar(c, fe_lstm_scope(d) + "kernel") + (long)C * 4 * U,
                         (long)4 * U, 1, 4 * U, U, U / 8, (int)TF_EFWD, U, c->fTWf.as<__bf16>() + (long)d * 4 * U * U);
    for (int d = 0; d < 2; ++d)  // zero initial h
      TT2_HIP(hipMemsetAsync(c->fHSh.as<__bf16>() + (long)d * (T + 1) * Bp * U, 0, 2 * (size_t)Bp * U, s));
    TrFused e{};
    e.Wt = c->fTWf.as<__bf16>(); e.wdir = (long)4 * U * U; e.K = U; e.B = B; e.H = U; e.T = T; e.lens = lens;
    e.zm = enczm; e.zo = f.zoneout; e.XP = c->fXP.as<float>(); e.GA = c->fGA.as<float>(); e.CN = c->fCN.as<float>();
    e.CS = c->fCS.as<float>(); e.HS = c->fHS.as<float>(); e.ENC = c->fENC.as<float>(); e.HSh = c->fHSh.as<__bf16>();
    e.adir = (T + 1) * Bp * U;
    for (int t = 0; t < T; ++t) {
      e.t = t;
      hipLaunchKernelGGL(k_tr_fused<TF_EFWD>, dim3(2 * 2 * U / 8), dim3(TLG_NT), 0, s, e);
    }
  } else {
    for (int t = 0; t < T; ++t) {
      for (int d = 0; d < 2; ++d)
        tr_gemm(B, 4 * U, U, c->fHS.as<float>() + ((long)d * (T + 1) + t) * B * U, U,
                pvar(c, fe_lstm_scope(d) + "kernel") + (long)C * 4 * U, 4 * U, c->fGZ.as<float>() + (long)d * B * 4 * U,
                4 * U, s);
      l.t = t;
      fe_lstm_cell(l, s);
    }
  }
  // reference encoders (modules.py:9-64) + GST (tacotron.py:276-282)
  const int RD = f.reference_depth;
  int nbn = f.enc_conv_layers;
  for (int r = 0; r < c->f_nref; ++r) {
    const std::string rs = fe_ref_scope(c, r);
    int H = T_ref, W = c->NM, ci = 1;
    const float* x = refs[r];
    for (int i = 0; i < 6; ++i) {
      const std::string sc = rs + "conv2d_" + std::to_string(i) + "/";
      const int st = fe_ref_stride(c, i);
      const int fo = f.reference_filters[i], Ho = (H + st - 1) / st, Wo = (W + st - 1) / st;
      GemmArgs g;
      g.M = B * Ho * Wo; g.N = fo; g.K = 9 * ci; g.a_mode = A_CONV2D; g.A = x;
      g.H = H; g.Wd = W; g.C = ci; g.Ho = Ho; g.Wo = Wo; g.kh = 3; g.kw2 = 3; g.sh = st; g.sw = st;
      g.pt = std::max((Ho - 1) * st + 3 - H, 0) / 2; g.pl = std::max((Wo - 1) * st + 3 - W, 0) / 2;
      g.Bw = pvar(c, sc + fe_ref_conv(c, r) + "kernel"); g.ldb = fo; g.ldc = fo;
      g.bias = pvar(c, sc + fe_ref_conv(c, r) + "bias");
      const bool small = c->fe_direct && fe_conv2d_fwd_small_ok(ci, fo);  // first layer: direct kernel
      if (c->f_adain) {  // conv2d(..., batch_norm=False): conv + ReLU (modules.py:84-87)
        g.Cout = c->fRY[r][i].as<float>();
        g.act = ACT_RELU;
        if (small)
          fe_conv2d_fwd_small(x, g.Bw, g.bias, B, H, W, ci, Ho, Wo, fo, g.pt, g.pl, st, true, g.Cout, s, g_tr_prec == 2);
        else
          tr_gemm_run(g, s);
      } else {
        g.Cout = c->fRA[r][i].as<float>();
        if (small)
          fe_conv2d_fwd_small(x, g.Bw, g.bias, B, H, W, ci, Ho, Wo, fo, g.pt, g.pl, st, false, g.Cout, s, g_tr_prec == 2);
        else
          tr_gemm_run(g, s);
        float* mean = BN + (long)nbn * 2 * 512;
        float* var = mean + 512;
        fe_stats(c, c->fRA[r][i].as<float>(), g.M, fo, mean, var, s);
        fe_bn_relu_fwd(c->fRA[r][i].as<float>(), g.M, fo, mean, var, pvar(c, sc + "batch_normalization/gamma"),
                       pvar(c, sc + "batch_normalization/beta"), eps, c->fRY[r][i].as<float>(), s);
        ++nbn;
      }
      x = c->fRY[r][i].as<float>();
      H = Ho; W = Wo; ci = fo;
    }
    const int T2 = H, gin = W * ci;
    c->f_T2 = T2;
    if (c->f_adain) {
      // moments over (time, freq) per row and channel (modules.py:90-91); the speaker map (r = 1,
      // after the emotion stack r = 0) restyled into fADX, which alone feeds the GRU (:94-104)
      float* mv = c->fADM.as<float>() + (long)r * B * ci * 2;
      fe_ad_moments(x, B, T2 * W, ci, mv, s);
      if (r == 0) continue;
      fe_ad_mix(x, B, T2 * W, ci, mv, c->fADM.as<float>(), c->fADX.as<float>(), s);
      x = c->fADX.as<float>();
    }
    const float* kg = pvar(c, rs + "rnn/gru_cell/gates/kernel");
    const float* kcn = pvar(c, rs + "rnn/gru_cell/candidate/kernel");
    float* XG = c->fXG[r].as<float>();
    tr_gemm(B * T2, 2 * RD, gin, x, gin, kg, 2 * RD, XG, 3 * RD, s, pvar(c, rs + "rnn/gru_cell/gates/bias"));
    tr_gemm(B * T2, RD, gin, x, gin, kcn, RD, XG + 2 * RD, 3 * RD, s, pvar(c, rs + "rnn/gru_cell/candidate/bias"));
    TT2_HIP(hipMemsetAsync(c->fHG[r].p, 0, sizeof(float) * (size_t)B * RD, s));
    if (c->fe_gru_seq && fe_gru_seq_ok(B, RD))  // the whole recurrence in one work-group (fp32 MFMA)
      fe_gru_fwd_seq(XG, kg + (long)gin * 2 * RD, kcn + (long)gin * RD, B, T2, RD, c->fGR[r].as<float>(), c->fGU[r].as<float>(),
                     c->fGRH[r].as<float>(), c->fGCC[r].as<float>(), c->fHG[r].as<float>(), s, g_tr_prec == 2);
    for (int t = 0; t < (c->fe_gru_seq && fe_gru_seq_ok(B, RD) ? 0 : T2); ++t) {
      float* h = c->fHG[r].as<float>() + (long)t * B * RD;
      tr_gemm(B, 2 * RD, RD, h, RD, kg + (long)gin * 2 * RD, 2 * RD, c->fGG.as<float>(), 2 * RD, s);
      fe_gru_a(XG, c->fGG.as<float>(), c->fHG[r].as<float>(), B, T2, RD, t, c->fGR[r].as<float>(),
               c->fGU[r].as<float>(), c->fGRH[r].as<float>(), s);
      tr_gemm(B, RD, RD, c->fGRH[r].as<float>() + (long)t * B * RD, RD, kcn + (long)gin * RD, RD, c->fGC.as<float>(), RD,
              s);
      fe_gru_b(XG, c->fGC.as<float>(), c->fGU[r].as<float>(), B, T2, RD, t, c->fGCC[r].as<float>(),
               c->fHG[r].as<float>(), s);
    }
    tr_gemm(B, 128, RD, c->fHG[r].as<float>() + (long)T2 * B * RD, RD, pvar(c, rs + "dense/kernel"), 128,
            c->fREF[r].as<float>(), 128, s, pvar(c, rs + "dense/bias"), nullptr, 0, ACT_TANH);
    if (c->f_adain) {  // the speaker reference embedding is the style embedding (tacotron.py:269-272)
      hipLaunchKernelGGL(k_tr_rows_copy, dim3(nblk((long)B * 128)), dim3(256), 0, s, c->fREF[r].as<float>(), 128L,
                         (long)B, 128, c->fSTY.as<float>(), (long)(c->D - 2 * f.encoder_lstm_units),
                         (const float*)nullptr, 0L);
    } else if (f.use_gst) {
      fe_gst_fwd(fe_gst_args(c, r, B), s);
    } else {  // the reference embedding is the style embedding (tacotron.py:284-291)
      const int SW = c->D - 2 * f.encoder_lstm_units;
      hipLaunchKernelGGL(k_tr_rows_copy, dim3(nblk((long)B * 128)), dim3(256), 0, s, c->fREF[r].as<float>(), 128L,
                         (long)B, 128, c->fSTY.as<float>() + r * 128, (long)SW, (const float*)nullptr, 0L);
    }
  }
  fe_memory(c->fENC.as<float>(), c->fSTY.as<float>(), B, T, 2 * U, c->D - 2 * U, c->fMEM.as<float>(), s);
  c->f_ran = true;
}

// ---- style-embedding losses (tacotron.py:486-495, 812-820, 840-846; oracle style_emb_losses) ----------
// Style_Emb_Disc: logits = ref·W + b [B, n]; softmax_cross_entropy_with_logits against tf.one_hot(label)
// (out-of-range label: zero row -> loss 0, gradient 0), batch mean.  One work-group per row: the
// row's loss -> part[b], d logits = (softmax·Σy - y) / B -> DL, d ref += DL·Wᵀ -> XR.
__global__ __launch_bounds__(128) void k_fe_disc(const float* __restrict__ ref, const float* __restrict__ Wk,
                                                 const float* __restrict__ bk, const int* __restrict__ lab, int B,
                                                 int n, float* __restrict__ DL, float* __restrict__ XR,
                                                 float* __restrict__ part) {
  extern __shared__ float sd[];  // [128] ref row, [n] logits
  const int b = blockIdx.x, k = threadIdx.x;
  float* lg = sd + 128;
  sd[k] = ref[(long)b * 128 + k];
  __syncthreads();
  for (int j = k; j < n; j += 128) {
    float v = bk[j];
    for (int i = 0; i < 128; ++i) v = fmaf(sd[i], Wk[(long)i * n + j], v);
    lg[j] = v;
  }
  __syncthreads();
  const int y = lab[b];
  const bool hot = y >= 0 && y < n;
  if (k == 0) {  // serial over n (small): max, log-sum-exp, loss
    float mx = -INFINITY;
    for (int j = 0; j < n; ++j) mx = fmaxf(mx, lg[j]);
    double se = 0;
    for (int j = 0; j < n; ++j) se += exp((double)(lg[j] - mx));
    const float lse = mx + (float)log(se);
    part[b] = hot ? lse - lg[y] : 0.f;
    sd[128 + n] = lse;
  }
  __syncthreads();
  const float lse = sd[128 + n];
  for (int j = k; j < n; j += 128) {
    const float d = hot ? (expf(lg[j] - lse) - (j == y ? 1.f : 0.f)) / (float)B : 0.f;
    DL[(long)b * n + j] = d;
    lg[j] = d;
  }
  __syncthreads();
  float g = 0.f;
  for (int j = 0; j < n; ++j) g = fmaf(lg[j], Wk[(long)k * n + j], g);
  XR[(long)b * 128 + k] += g;
}
// d W[k][j] = Σ_b ref[b][k] DL[b][j], d b[j] = Σ_b DL[b][j] (written, not accumulated)
__global__ void k_fe_disc_wgrad(const float* __restrict__ ref, const float* __restrict__ DL, int B, int n,
                                float* __restrict__ dW, float* __restrict__ db) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 128 * n) {
    const int k = i / n, j = i % n;
    float v = 0.f;
    for (int b = 0; b < B; ++b) v = fmaf(ref[(long)b * 128 + k], DL[(long)b * n + j], v);
    dW[i] = v;
  } else if (i < 129 * n) {
    const int j = i - 128 * n;
    float v = 0.f;
    for (int b = 0; b < B; ++b) v += DL[(long)b * n + j];
    db[j] = v;
  }
}
// orthogonality loss w·||E·Sᵀ||_F: M = E·Sᵀ [B][B] (row b per work-group), Σ M² partials
__global__ __launch_bounds__(128) void k_fe_orthog_m(const float* __restrict__ E, const float* __restrict__ S, int B,
                                                     float* __restrict__ M, float* __restrict__ part) {
  __shared__ float e[128];
  __shared__ float s4[4];
  const int b = blockIdx.x, t = threadIdx.x;
  e[t] = E[(long)b * 128 + t];
  __syncthreads();
  float sq = 0.f;
  for (int jj = t; jj < B; jj += 128) {
    float v = 0.f;
    for (int i = 0; i < 128; ++i) v = fmaf(e[i], S[(long)jj * 128 + i], v);
    M[(long)b * B + jj] = v;
    sq += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
  if ((t & 63) == 0) s4[t >> 6] = sq;
  __syncthreads();
  if (t == 0) part[b] = s4[0] + s4[1];
}
// loss = w·||M|| -> red[0]; d E = (w/||M||)·M·S -> XE, d S = (w/||M||)·Mᵀ·E -> XS (accumulated);
// blocks [0, B) rows of d E, [B, 2B) rows of d S.  ||M|| = 0: TF's norm gradient is NaN there; 0 here.
__global__ __launch_bounds__(128) void k_fe_orthog_g(const float* __restrict__ E, const float* __restrict__ S,
                                                     const float* __restrict__ M, int B, float w,
                                                     const float* __restrict__ n2, float* __restrict__ red,
                                                     float* __restrict__ XE, float* __restrict__ XS) {
  const int r = blockIdx.x, k = threadIdx.x;
  const float nrm = sqrtf(n2[0]);
  if (r == 0 && k == 0) red[0] = w * nrm;
  const float coef = nrm > 0.f ? w / nrm : 0.f;
  float g = 0.f;
  if (r < B) {
    for (int j = 0; j < B; ++j) g = fmaf(M[(long)r * B + j], S[(long)j * 128 + k], g);
    XE[(long)r * 128 + k] += coef * g;
  } else {
    const int j = r - B;
    for (int b = 0; b < B; ++b) g = fmaf(M[(long)b * B + j], E[(long)b * 128 + k], g);
    XS[(long)j * 128 + k] += coef * g;
  }
}

// The style-embedding losses' gradients into the refnet outputs (sXREF[r]) and the classifier
// weights; losses -> red[5] (emt), red[6] (spk), red[7] (orthogonality).  Before the refnet backward.
static void tr_style_losses(tt2_train_ctx* c, hipStream_t s) {
  const auto& f = c->cfg;
  const int B = c->B;
  float* red = c->red.as<float>();
  float* XR = c->sXREF.as<float>();
  TT2_HIP(hipMemsetAsync(XR, 0, sizeof(float) * (size_t)2 * B * 128, s));
  TT2_HIP(hipMemsetAsync(red + 5, 0, sizeof(float) * 3, s));
  for (int r = 0; r < c->f_nref; ++r) {
    const int n = r == 0 ? f.n_emt : f.n_spk;
    if (n <= 0) continue;
    const std::string sd = vn(r == 0 ? "style_disc_emt/dense/" : "style_disc_spk/dense/");
    hipLaunchKernelGGL(k_fe_disc, dim3(B), dim3(128), sizeof(float) * (129 + n), s, c->fREF[r].as<float>(),
                       pvar(c, sd + "kernel"), pvar(c, sd + "bias"), c->sLAB.as<int>() + r * B, B, n, c->sDL.as<float>(),
                       XR + (long)r * B * 128, c->part.as<float>());
    hipLaunchKernelGGL(k_tr_sum_final, dim3(1), dim3(256), 0, s, c->part.as<float>(), B, 1.0f / B, red + 5 + r, 0);
    hipLaunchKernelGGL(k_fe_disc_wgrad, dim3((129 * n + 255) / 256), dim3(256), 0, s, c->fREF[r].as<float>(),
                       c->sDL.as<float>(), B, n, gvar(c, sd + "kernel"), gvar(c, sd + "bias"));
  }
  if (f.orthog_weight > 0.f && c->f_nref == 2) {
    hipLaunchKernelGGL(k_fe_orthog_m, dim3(B), dim3(128), 0, s, c->fREF[0].as<float>(), c->fREF[1].as<float>(), B,
                       c->sOM.as<float>(), c->part.as<float>());
    hipLaunchKernelGGL(k_tr_sum_final, dim3(1), dim3(256), 0, s, c->part.as<float>(), B, 1.0f, red + 8, 0);
    hipLaunchKernelGGL(k_fe_orthog_g, dim3(2 * B), dim3(128), 0, s, c->fREF[0].as<float>(), c->fREF[1].as<float>(),
                       c->sOM.as<float>(), B, f.orthog_weight, red + 8, red + 7, XR, XR + (long)B * 128);
  }
  TT2_HIP(hipGetLastError());
}

static bool tr_style_on(const tt2_train_ctx* c) {
  return c->cfg.n_emt > 0 || (c->f_nref == 2 && (c->cfg.n_spk > 0 || c->cfg.orthog_weight > 0.f));
}

static void tr_front_backward(tt2_train_ctx* c, const int* ids, const int* lens, const float* const* refs, int T_ref,
                              const uint8_t* encm, const uint8_t* enczm, int T, hipStream_t s) {
  const auto& f = c->cfg;
  const int B = c->B, E = f.embedding_dim, C = f.enc_conv_channels, K = f.enc_conv_kernel, U = f.encoder_lstm_units;
  const int D = c->D, RD = f.reference_depth, SW = D - 2 * U;
  const long M = (long)B * T;
  float* BN = c->fBN.as<float>();
  float* WT = c->fWT.as<float>();
  float* FB = c->fFBUF.as<float>();
  // memory assembly: style gradient = Σ_t over the (length-masked) d memory rows
  fe_style_grad(c->DMEM.as<float>(), B, T, D, 2 * U, c->fDSTY.as<float>(), s);
  const bool style_on = tr_style_on(c);
  if (style_on) tr_style_losses(c, s);
  // conv2d stack r backward from d map `din` (conv -> BN -> ReLU per layer; AdaIN: conv -> ReLU)
  const bool fe_direct = c->fe_direct;
  auto conv_bwd = [&](int r, const float* din) {
    const std::string rs = fe_ref_scope(c, r);
    float* dY = c->fDY.as<float>();
    int dims[7][3];
    {
      int H = T_ref, W = c->NM, ci = 1;
      for (int i = 0; i < 6; ++i) {
        dims[i][0] = H; dims[i][1] = W; dims[i][2] = ci;
        const int st = fe_ref_stride(c, i);
        H = (H + st - 1) / st; W = (W + st - 1) / st; ci = f.reference_filters[i];
      }
      dims[6][0] = H; dims[6][1] = W; dims[6][2] = ci;
    }
    for (int i = 5; i >= 0; --i) {
      const int nbn = f.enc_conv_layers + 6 * r + i;  // forward order: encoder convs, then refnet r's layers
      const std::string sc = rs + "conv2d_" + std::to_string(i) + "/", ly = fe_ref_conv(c, r);
      const int H = dims[i][0], W = dims[i][1], ci = dims[i][2], Ho = dims[i + 1][0], Wo = dims[i + 1][1];
      const int fo = f.reference_filters[i], st = fe_ref_stride(c, i);
      const long Mi = (long)B * Ho * Wo;
      float* dYr = c->fDY2.as<float>();
      fe_relu_mask(i == 5 ? din : dY, c->fRY[r][i].as<float>(), Mi * fo, dYr, s);
      float* dz = dYr;
      if (!c->f_adain) {
        const float* mean = BN + (long)nbn * 2 * 512;
        const float* var = mean + 512;
        dz = c->fDZc.as<float>();
        fe_bn_bwd(c, dYr, nullptr, c->fRA[r][i].as<float>(), Mi, fo, mean, var, sc, 0, dYr, dz, s);
      }
      tr_colsum(c, dz, Mi, fo, fo, gvar(c, sc + ly + "bias"), s);
      const int pt = std::max((Ho - 1) * st + 3 - H, 0) / 2, pl = std::max((Wo - 1) * st + 3 - W, 0) / 2;
      const float* xin = i == 0 ? refs[r] : c->fRY[r][i - 1].as<float>();
      // kernel gradient: direct (k_fe_conv2d_dw: patches staged in LDS, fp32 FMA, partial rows summed
      // by tr_colsum) where its register / LDS budget takes the channel counts, else the im2colᵀ
      // columns + GEMM (gemm_bf16_kc with the im2colᵀ gathered into bf16 measured 458 us per layer
      // against 525 + ~60 for the fp32 columns + gemm_x3_kernel: its 256-wide N tile is 8x idle at fo = 32)
      if (fe_direct && fe_conv2d_dw_ok(ci, fo)) {
        const int rows = fe_conv2d_dw(xin, dz, B, H, W, ci, Ho, Wo, fo, pt, pl, st, FB, (long)(c->fFBUF.bytes / sizeof(float)),
                                      s);
        tr_colsum(c, FB, rows, 9 * ci * fo, 9L * ci * fo, gvar(c, sc + ly + "kernel"), s);
      } else {
        fe_im2col2d_t(xin, B, H, W, ci, Ho, Wo, pt, pl, FB, Mi, s, st);
        tr_gemm(9 * ci, fo, (int)Mi, FB, Mi, dz, fo, gvar(c, sc + ly + "kernel"), fo, s);
      }
      if (i > 0) {
        if (fe_direct && fe_conv2d_dx_ok(ci, W, Ho, Wo, fo, st)) {  // input gradient as a gather over the taps (k_fe_conv2d_dx)
          fe_conv2d_dx(dz, pvar(c, sc + ly + "kernel"), B, H, W, ci, Ho, Wo, fo, pt, pl, st, dY, s);
        } else {
          tr_transpose(pvar(c, sc + ly + "kernel"), 9L * ci, fo, fo, WT, 9L * ci, s);  // [fo][9ci]
          tr_gemm((int)Mi, 9 * ci, fo, dz, fo, WT, 9 * ci, FB, 9 * ci, s);
          fe_col2im2d(FB, B, H, W, ci, Ho, Wo, pt, pl, dY, s, st);
        }
      }
    }
  };
  for (int r = c->f_adain ? 1 : 0; r < c->f_nref; ++r) {
    const std::string rs = fe_ref_scope(c, r), m = fe_mh_scope(r);
    if (!f.use_gst || c->f_adain) {  // d ref = d style slice (+ style-loss terms)
      hipLaunchKernelGGL(k_tr_rows_copy, dim3(nblk((long)B * 128)), dim3(256), 0, s,
                         c->fDSTY.as<float>() + (c->f_adain ? 0 : r * 128),
                         (long)SW, (long)B, 128, c->fdREF.as<float>(), 128L,
                         style_on ? (const float*)(c->sXREF.as<float>() + (long)r * B * 128) : (const float*)nullptr,
                         128L);
    } else {
    const FeGst ga = fe_gst_args(c, r, B);
    fe_gst_bwd(ga, s);
    const int ntok = ga.ntok, tokd = ga.tokd, A = ga.A, dh = A / ga.heads;
    float* sum = c->fGsum.as<float>();
    tr_colsum(c, ga.pdkk, B, ntok * A, (long)ntok * A, sum, s);
    tr_colsum(c, ga.pdv, B, ntok * tokd, (long)ntok * tokd, sum + ntok * A, s);
    tr_colsum(c, ga.pdnv, B, dh, dh, sum + ntok * A + ntok * tokd, s);
    tr_colsum(c, ga.pdbb, B, dh, dh, sum + ntok * A + ntok * tokd + dh, s);
    fe_gst_final(ga, sum, sum + ntok * A, sum + ntok * A + ntok * tokd, sum + ntok * A + ntok * tokd + dh,
                 gvar(c, m + "conv1d_1/kernel"), gvar(c, m + "conv1d_1/bias"),
                 gvar(c, vn(r == 0 ? "style_tokens_emt" : "style_tokens_spk")), gvar(c, m + "attention_v"),
                 gvar(c, m + "attention_g"), gvar(c, m + "attention_b"), s);
    // query conv1d (1x1): d Wq = refᵀ dq, d bq, d ref = dq Wqᵀ
    tr_transpose(c->fREF[r].as<float>(), B, 128, 128, WT, B, s);
    tr_gemm(128, A, B, WT, B, ga.dq, A, gvar(c, m + "conv1d/kernel"), A, s);
    tr_colsum(c, ga.dq, B, A, A, gvar(c, m + "conv1d/bias"), s);
    tr_transpose(pvar(c, m + "conv1d/kernel"), 128, A, A, WT, 128, s);
    tr_gemm(B, 128, A, ga.dq, A, WT, 128, c->fdREF.as<float>(), 128, s, nullptr,
            style_on ? c->sXREF.as<float>() + (long)r * B * 128 : nullptr, 128);  // + style-loss terms
    }
    // dense tanh (modules.py:63)
    fe_tanh_bwd(c->fdREF.as<float>(), c->fREF[r].as<float>(), (long)B * 128, c->fDZD.as<float>(), s);
    const int T2 = c->f_T2;
    const float* hT = c->fHG[r].as<float>() + (long)T2 * B * RD;
    tr_transpose(hT, B, RD, RD, WT, B, s);
    tr_gemm(RD, 128, B, WT, B, c->fDZD.as<float>(), 128, gvar(c, rs + "dense/kernel"), 128, s);
    tr_colsum(c, c->fDZD.as<float>(), B, 128, 128, gvar(c, rs + "dense/bias"), s);
    tr_transpose(pvar(c, rs + "dense/kernel"), RD, 128, 128, WT, RD, s);
    tr_gemm(B, RD, 128, c->fDZD.as<float>(), 128, WT, RD, c->fDH.as<float>(), RD, s);
    // GRU BPTT (TF1 GRUCell): recurrent weight transposes once
    const int gin = c->f_gin;
    const float* kg = pvar(c, rs + "rnn/gru_cell/gates/kernel");
    const float* kcn = pvar(c, rs + "rnn/gru_cell/candidate/kernel");
    float* WghT = WT;                       // [2RD][RD]
    float* WchT = WT + 2L * RD * RD;        // [RD][RD]
    const bool gseq = c->fe_gru_seq && fe_gru_seq_ok(B, RD);
    if (gseq) {  // the whole reverse recurrence in one work-group (fp32 MFMA)
      fe_gru_bwd_seq(kg + (long)gin * 2 * RD, kcn + (long)gin * RD, c->fGR[r].as<float>(), c->fGU[r].as<float>(),
                     c->fGCC[r].as<float>(), c->fHG[r].as<float>(), B, T2, RD, c->fDH.as<float>(), c->fDCP.as<float>(),
                     c->fDGP.as<float>(), s, g_tr_prec == 2);
    } else {
      tr_transpose(kg + (long)gin * 2 * RD, RD, 2 * RD, 2 * RD, WghT, RD, s);
      tr_transpose(kcn + (long)gin * RD, RD, RD, RD, WchT, RD, s);
    }
    for (int t = gseq ? -1 : T2 - 1; t >= 0; --t) {
      fe_gru_bwd_a(c->fDH.as<float>(), c->fGU[r].as<float>(), c->fGCC[r].as<float>(), c->fHG[r].as<float>(), B, RD, t,
                   c->fDCP.as<float>(), c->fDHA.as<float>(), s);
      tr_gemm(B, RD, RD, c->fDCP.as<float>() + (long)t * B * RD, RD, WchT, RD, c->fDRH.as<float>(), RD, s);
      fe_gru_bwd_b(c->fDRH.as<float>(), c->fGR[r].as<float>(), c->fGU[r].as<float>(), c->fHG[r].as<float>(),
                   c->fGCC[r].as<float>(), c->fDH.as<float>(), B, RD, t, c->fDGP.as<float>(), c->fDHA.as<float>(), s);
      tr_gemm(B, RD, 2 * RD, c->fDGP.as<float>() + (long)t * B * 2 * RD, 2 * RD, WghT, RD, c->fDH.as<float>(), RD, s,
              nullptr, c->fDHA.as<float>(), RD);
    }
    // recurrent weight gradients over all steps: d Wg_h = Σ h(t)ᵀ dGP(t), d Wc_h = Σ (r h)(t)ᵀ dCP(t)
    const long R2 = (long)T2 * B;
    tr_transpose(c->fHG[r].as<float>(), R2, RD, RD, FB, R2, s);
    tr_gemm(RD, 2 * RD, (int)R2, FB, R2, c->fDGP.as<float>(), 2 * RD, gvar(c, rs + "rnn/gru_cell/gates/kernel") +
            (long)gin * 2 * RD, 2 * RD, s);
    tr_transpose(c->fGRH[r].as<float>(), R2, RD, RD, FB, R2, s);
    tr_gemm(RD, RD, (int)R2, FB, R2, c->fDCP.as<float>(), RD, gvar(c, rs + "rnn/gru_cell/candidate/kernel") +
            (long)gin * RD, RD, s);
    // input side over all (n, t) rows: DXG = [dGP | dCP] in (n, t) order
    fe_gru_dxg(c->fDGP.as<float>(), c->fDCP.as<float>(), B, T2, RD, c->fDXG.as<float>(), s);
    const float* x6 = c->f_adain ? c->fADX.as<float>() : c->fRY[r][5].as<float>();
    tr_transpose(x6, R2, gin, gin, FB, R2, s);
    tr_gemm(gin, 2 * RD, (int)R2, FB, R2, c->fDXG.as<float>(), 3 * RD, gvar(c, rs + "rnn/gru_cell/gates/kernel"),
            2 * RD, s);
    tr_gemm(gin, RD, (int)R2, FB, R2, c->fDXG.as<float>() + 2 * RD, 3 * RD,
            gvar(c, rs + "rnn/gru_cell/candidate/kernel"), RD, s);
    tr_colsum(c, c->fDXG.as<float>(), R2, 2 * RD, 3 * RD, gvar(c, rs + "rnn/gru_cell/gates/bias"), s);
    tr_colsum(c, c->fDXG.as<float>() + 2 * RD, R2, RD, 3 * RD, gvar(c, rs + "rnn/gru_cell/candidate/bias"), s);
    float* dY = c->fDY.as<float>();
    tr_transpose(kg, gin, 2 * RD, 2 * RD, WT, gin, s);  // [2RD][gin]
    tr_gemm((int)R2, gin, 2 * RD, c->fDXG.as<float>(), 3 * RD, WT, gin, dY, gin, s);
    tr_transpose(kcn, gin, RD, RD, WT, gin, s);
    tr_gemm((int)R2, gin, RD, c->fDXG.as<float>() + 2 * RD, 3 * RD, WT, gin, dY, gin, s, nullptr, dY, gin);
    if (!c->f_adain) {
      conv_bwd(r, dY);
      continue;
    }
    // AdaIN: the restyle's backward splits d map into the speaker map's gradient (in place) and the
    // emotion map's (through its moments), then both stacks run backward
    const int C6 = f.reference_filters[5], HW = T2 * (gin / C6);
    fe_ad_mix_bwd(dY, c->fRY[1][5].as<float>(), c->fRY[0][5].as<float>(), B, HW, C6, c->fADM.as<float>() + (long)B * C6 * 2,
                  c->fADM.as<float>(), c->fADS.as<float>(), dY, c->fDYE.as<float>(), s);
    conv_bwd(1, dY);  // (din is read by the top layer's ReLU mask before any col2im writes dY)
    conv_bwd(0, c->fDYE.as<float>());
  }
  // BiLSTM BPTT (the decoder's DMEM rows carry d enc_out in columns [0, 2U))
  for (int d = 0; d < 2; ++d) {
    const float* k = pvar(c, fe_lstm_scope(d) + "kernel");
    tr_transpose(k + (long)C * 4 * U, U, 4 * U, 4 * U, c->fLWhT.as<float>() + (long)d * 4 * U * U, U, s);
    tr_transpose(k, C, 4 * U, 4 * U, c->fLWxT.as<float>() + (long)d * 4 * U * C, C, s);
  }
  TT2_HIP(hipMemsetAsync(c->fDHC.p, 0, c->fDHC.bytes, s));
  TT2_HIP(hipMemsetAsync(c->fDCC.p, 0, c->fDCC.bytes, s));
  FeLstm l{};
  l.GA = c->fGA.as<float>(); l.CN = c->fCN.as<float>(); l.CS = c->fCS.as<float>(); l.HS = c->fHS.as<float>();
  l.zm = enczm; l.lens = lens; l.B = B; l.T = T; l.U = U; l.zo = f.zoneout;
  l.DENC = c->DMEM.as<float>(); l.ld_denc = D; l.DZ = c->fDZ.as<float>(); l.DHC = c->fDHC.as<float>();
  l.DCC = c->fDCC.as<float>(); l.DHP = c->fDHP.as<float>();
  if (fe_enc_fused(c)) {  // d h carried = dZ(t+1)·Wh^T + its direct part, fused with the cell backward
    const long Bp = (B + 31) & ~31L;
    for (int d = 0; d < 2; ++d)
      hipLaunchKernelGGL(k_tr_tf_weights_f32, dim3(1024), dim3(256), 0, s, pvar(c, fe_lstm_scope(d) + "kernel") + (long)C * 4 * U,
                         (long)4 * U, 0, U, 4 * U, U / 32, (int)TF_PLAIN, U, c->fTWb.as<__bf16>() + (long)d * 4 * U * U);
    TT2_HIP(hipMemsetAsync(c->fDZh.p, 0, c->fDZh.bytes, s));  // dZ(T) = 0
    TT2_HIP(hipMemsetAsync(c->fDHP.p, 0, c->fDHP.bytes, s));
    TrFused e{};
    e.Wt = c->fTWb.as<__bf16>(); e.wdir = (long)4 * U * U; e.K = 4 * U; e.B = B; e.H = U; e.T = T; e.lens = lens;
    e.zm = enczm; e.zo = f.zoneout; e.GA = c->fGA.as<float>(); e.CN = c->fCN.as<float>(); e.CS = c->fCS.as<float>();
    e.DENC = c->DMEM.as<float>(); e.ld_denc = D; e.DZ = c->fDZ.as<float>(); e.DCC = c->fDCC.as<float>();
    e.DHP = c->fDHP.as<float>(); e.DZh = c->fDZh.as<__bf16>(); e.adir = 2 * Bp * 4 * U;
    for (int t = T - 1; t >= 0; --t) {
      e.t = t;
      hipLaunchKernelGGL(k_tr_fused<TF_EBWD>, dim3(2 * 2 * U / 32), dim3(TLG_NT), 0, s, e);
    }
  } else {
    for (int t = T - 1; t >= 0; --t) {
      l.t = t;
      fe_lstm_cell_bwd(l, s);
      for (int d = 0; d < 2; ++d)
        tr_gemm(B, U, 4 * U, c->fDZ.as<float>() + ((long)d * T + t) * B * 4 * U, 4 * U,
                c->fLWhT.as<float>() + (long)d * 4 * U * U, U, c->fDHC.as<float>() + (long)d * B * U, U, s, nullptr,
                c->fDHP.as<float>() + (long)d * B * U, U);
    }
  }
  for (int d = 0; d < 2; ++d) {  // recurrent weights: Σ_t HS(t)ᵀ DZ(t); biases
    const long R = (long)T * B;
    tr_transpose(c->fHS.as<float>() + (long)d * (T + 1) * B * U, R, U, U, FB, R, s);
    tr_gemm(U, 4 * U, (int)R, FB, R, c->fDZ.as<float>() + (long)d * T * B * 4 * U, 4 * U,
            gvar(c, fe_lstm_scope(d) + "kernel") + (long)C * 4 * U, 4 * U, s);
    tr_colsum(c, c->fDZ.as<float>() + (long)d * T * B * 4 * U, R, 4 * U, 4 * U, gvar(c, fe_lstm_scope(d) + "bias"), s);
  }
  fe_lstm_dxp(c->fDZ.as<float>(), lens, B, T, U, c->fdXP.as<float>(), s);
  const float* X3 = c->fEY[f.enc_conv_layers].as<float>();
  tr_transpose(X3, M, C, C, FB, M, s);
  float* dxn = c->fdA.as<float>();
  float* dxo = c->fdB.as<float>();
  for (int d = 0; d < 2; ++d) {
    tr_gemm(C, 4 * U, (int)M, FB, M, c->fdXP.as<float>() + d * 4 * U, 8 * U, gvar(c, fe_lstm_scope(d) + "kernel"),
            4 * U, s);
    tr_gemm((int)M, C, 4 * U, c->fdXP.as<float>() + d * 4 * U, 8 * U, c->fLWxT.as<float>() + (long)d * 4 * U * C, C,
            dxn, C, s, nullptr, d ? dxn : nullptr, C);
  }
  // encoder convolutions backward (dropout -> BN -> ReLU -> conv)
  for (int i = f.enc_conv_layers - 1; i >= 0; --i) {
    const std::string sc = fe_conv_scope(i + 1);
    const float* mean = BN + (long)i * 2 * 512;
    const float* var = mean + 512;
    float* dz = c->fDZc.as<float>();
    const bool bplanes = c->fePl.p && g_tr_prec == 2;
    __bf16* bpl = reinterpret_cast<__bf16*>(c->fePl.p);
    fe_bn_bwd(c, dxn, encm ? encm + (long)i * M * C : nullptr, c->fEA[i].as<float>(), M, C, mean, var, sc, 2,
              c->fDY.as<float>(), dz, s, bplanes ? bpl : nullptr, T);
    tr_colsum(c, dz, M, C, C, gvar(c, sc + "conv1d/bias"), s);
    const int cin = i == 0 ? E : C, pad = (K - 1) / 2;
    const float* xin = i == 0 ? c->fEX.as<float>() : c->fEY[i].as<float>();
    if (c->blas_on && g_tr_prec == 2 && 2.0 * K * cin * (double)C * M >= kTrBigMinFlops) {
      KcConvA cv;  // im2colᵀ gathered straight into gemm_bf16_kc's bf16 operand copy
      cv.x = xin; cv.xs_b = (long)T * cin; cv.xs_t = cin; cv.B = B; cv.T = T; cv.C = cin; cv.kw = K; cv.pad = pad;
      gemm_bf16_kc(K * cin, C, (int)M, nullptr, 0, dz, C, gvar(c, sc + "conv1d/kernel"), C, c->blasA, c->blasB,
                   c->blasP, s, false, &cv);
      ++c->blas_calls;
    } else {
      hipLaunchKernelGGL(k_pn_im2col_t, dim3(nblk((long)K * cin * M)), dim3(256), 0, s, xin, (long)T * cin, (long)cin,
                         B, T, cin, K, pad, FB, M);
      tr_gemm(K * cin, C, (int)M, FB, M, dz, C, gvar(c, sc + "conv1d/kernel"), C, s);
    }
    hipLaunchKernelGGL(k_pn_flip, dim3(nblk((long)K * cin * C)), dim3(256), 0, s, pvar(c, sc + "conv1d/kernel"), K, cin,
                       C, WT);
    if (bplanes) {  // input gradient: conv of the dz planes with the flipped kernel
      __bf16* bwt = reinterpret_cast<__bf16*>(c->feWt.p);
      kc_transpose_bf16(WT, K * C, cin, cin, bwt, K * C, (cin + 255) / 256 * 256, s);
      conv_bf16_planes(bpl, C, B, T, K, bwt, (long)K * C, cin, nullptr, ACT_NONE, dxo, cin, s);
    } else {
      GemmArgs g;
      g.a_mode = A_CONV1D; g.M = (int)M; g.N = cin; g.T = T; g.kw = K; g.pad = K - 1 - pad;
      g.A = dz; g.C = C; g.xs_b = (long)T * C; g.xs_t = C; g.K = K * C;
      g.Bw = WT; g.ldb = cin; g.Cout = dxo; g.ldc = cin;
      tr_gemm_run(g, s);
    }
    std::swap(dxn, dxo);
  }
  fe_embed_bwd(ids, dxn, M, E, f.n_symbols, gvar(c, vn("inputs_embedding")), s, FB,
               (long)(c->fFBUF.bytes / sizeof(float)));  // FB is free after the conv loop
}


static void tr_apply(tt2_train_ctx* c, float lr, int global_step, hipStream_t s) {
  float* red = c->red.as<float>();
  if (c->cfg.postnet && c->pn_ran) {  // BN UPDATE_OPS run with the optimizer (tacotron.py:1088-1090)
    for (int i = 0; i < c->PL; ++i) {
      const std::string sc = pn_scope(i + 1) + "batch_normalization/";
      hipLaunchKernelGGL(k_pn_moving, dim3((c->PC + 255) / 256), dim3(256), 0, s, pvar(c, sc + "moving_mean"),
                         pvar(c, sc + "moving_variance"), c->BNM.as<float>() + (long)i * c->PC,
                         c->BNV.as<float>() + (long)i * c->PC, c->PC, c->cfg.bn_momentum, c->grads + c->total);
    }
    c->pn_ran = false;
  }
  if (c->cfg.frontend && c->f_ran) {  // front-end BN UPDATE_OPS (encoder convs, then refnet convs)
    int nbn = 0;
    auto upd = [&](const std::string& sc, int C) {
      const float* st = c->fBN.as<float>() + (long)nbn * 2 * 512;
      hipLaunchKernelGGL(k_pn_moving, dim3((C + 255) / 256), dim3(256), 0, s, pvar(c, sc + "batch_normalization/moving_mean"),
                         pvar(c, sc + "batch_normalization/moving_variance"), st, st + 512, C, c->cfg.bn_momentum,
                         c->grads + c->total);
      ++nbn;
    };
    for (int i = 0; i < c->cfg.enc_conv_layers; ++i) upd(fe_conv_scope(i + 1), c->cfg.enc_conv_channels);
    for (int r = 0; r < c->f_nref && !c->f_adain; ++r)  // (AdaIN's refnet has no batch norm)
      for (int i = 0; i < 6; ++i) upd(fe_ref_scope(c, r) + "conv2d_" + std::to_string(i) + "/", c->cfg.reference_filters[i]);
    c->f_ran = false;
  }
  hipLaunchKernelGGL(k_tr_sumsq, dim3(TR_SUMSQ_BLOCKS), dim3(256), 0, s, c->grads, c->total, c->part.as<float>(),
                     (int)(reinterpret_cast<uintptr_t>(c->grads) % 16 == 0));
  hipLaunchKernelGGL(k_tr_sum_final, dim3(1), dim3(256), 0, s, c->part.as<float>(), TR_SUMSQ_BLOCKS, 1.f, red + 3, 1);
  const double b1 = c->cfg.adam_beta1, b2 = c->cfg.adam_beta2;
  const int t = std::max(1, global_step);
  const float lr_t = (float)(lr * std::sqrt(1.0 - std::pow(b2, t)) / (1.0 - std::pow(b1, t)));
  hipLaunchKernelGGL(k_tr_adam, dim3(nblk(c->total)), dim3(256), 0, s, c->params.as<float>(), c->grads,
                     c->adam_m.as<float>(), c->adam_v.as<float>(), c->total, red + 3, c->cfg.clip_norm,
                     c->cfg.adam_beta1, c->cfg.adam_beta2, c->cfg.adam_epsilon, lr_t);
}

}  // namespace tt2

// device -> host read-back ordered after the producing stream (see tt2_train_losses)
static void tr_d2h(tt2_train_ctx* c, void* dst, const void* src, size_t bytes) {
  if (c->last_stream) {
    TT2_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->last_stream));
    TT2_HIP(hipStreamSynchronize(c->last_stream));
  } else {
    TT2_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  }
}

// ---- C ABI -------------------------------------------------------------------------------------
extern "C" {

void tt2_train_default_config(tt2_train_config* c, int batch, int max_T_in, int max_T_out) {
  std::memset(c, 0, sizeof(*c));
  c->batch = batch;
  c->max_T_in = max_T_in;
  c->max_T_out = max_T_out;
  c->memory_dim = 1024;
  c->num_mels = 80;
  c->prenet_units = 256;
  c->decoder_lstm_units = 1024;
  c->attention_dim = 128;
  c->attention_filters = 32;
  c->attention_kernel = 31;
  c->zoneout = 0.1f;
  c->reg_weight = 1e-6f;
  c->adam_beta1 = 0.9f;
  c->adam_beta2 = 0.999f;
  c->adam_epsilon = 1e-6f;
  c->clip_norm = 1.0f;
  c->precision = 0;
  c->clip_outputs = 1;
  c->clip_lo = -4.1f;
  c->clip_hi = 4.0f;
  c->postnet = 0;
  c->postnet_layers = 5;
  c->postnet_channels = 512;
  c->postnet_kernel = 5;
  c->bn_momentum = 0.99f;
  c->bn_eps = 1e-3f;
  c->frontend = 0;
  c->n_symbols = 66;
  c->embedding_dim = 512;
  c->enc_conv_layers = 3;
  c->enc_conv_kernel = 5;
  c->enc_conv_channels = 512;
  c->encoder_lstm_units = 256;
  c->emt_only = 0;
  c->n_emt = 0;
  c->n_spk = 0;
  c->orthog_weight = 0.f;
  c->use_gst = 1;
  c->num_gst = 10;
  c->num_heads = 4;
  c->style_embed_depth = 256;
  c->style_att_dim = 128;
  c->reference_depth = 128;
  const int rf[6] = {32, 32, 64, 64, 128, 128};
  for (int i = 0; i < 6; ++i) c->reference_filters[i] = rf[i];
  c->max_T_ref = max_T_out;
  c->mask_decoder = 0;
  c->pos_weight = 1.0f;
  c->adain = 0;
  c->smoothing = 0;
  c->outputs_per_step = 1;
}

tt2_status tt2_train_set_target_lengths(tt2_train_ctx* c, const int32_t* lengths) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    if (!lengths) {
      c->has_tlen = false;
      return;
    }
    long sum = 0;
    int mx = 0;
    for (int b = 0; b < c->B; ++b) {
      TT2_CHECK(lengths[b] >= 1 && lengths[b] <= c->Tm, TT2_ERR_SHAPE_MISMATCH,
                "target length out of [1, max_T_out]");
      sum += lengths[b];
      mx = std::max(mx, (int)lengths[b]);
    }
    TT2_HIP(hipSetDevice(c->dev));
    // TLEN is read by the loss kernels of a forward_backward that may still be running on the
    // caller's (non-blocking) stream: let it finish before the lengths change under it
    if (c->last_stream) TT2_HIP(hipStreamSynchronize(c->last_stream));
    TT2_HIP(hipMemcpy(c->TLEN.p, lengths, sizeof(int) * (size_t)c->B, hipMemcpyHostToDevice));
    c->has_tlen = true;
    c->tlen_sum = sum;
    c->tlen_max = mx;
  });
}

tt2_status tt2_train_set_style_labels(tt2_train_ctx* c, const int32_t* emt_labels, const int32_t* spk_labels) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    if (!emt_labels && !spk_labels) {
      c->has_labels = false;
      return;
    }
    TT2_CHECK(emt_labels && (spk_labels || c->f_nref == 1), TT2_ERR_INVALID_ARG,
              "emotion labels (and speaker labels unless emt_only) required");
    std::vector<int> lab((size_t)2 * c->B, -1);
    for (int b = 0; b < c->B; ++b) {
      lab[b] = emt_labels[b];
      if (spk_labels) lab[c->B + b] = spk_labels[b];
    }
    TT2_HIP(hipSetDevice(c->dev));
    if (c->last_stream) TT2_HIP(hipStreamSynchronize(c->last_stream));  // a running step reads them
    TT2_HIP(hipMemcpy(c->sLAB.p, lab.data(), sizeof(int) * lab.size(), hipMemcpyHostToDevice));
    c->has_labels = true;
  });
}

tt2_status tt2_train_style_losses(tt2_train_ctx* c, float* out3) {
  return guard([&] {
    TT2_CHECK(c && out3, TT2_ERR_INVALID_ARG, "null argument");
    TT2_HIP(hipSetDevice(c->dev));
    if (!c->cfg.frontend || !tr_style_on(c) || !c->last_stream) {
      out3[0] = out3[1] = out3[2] = 0.f;
      return;
    }
    TT2_HIP(hipMemcpyAsync(out3, c->red.as<float>() + 5, sizeof(float) * 3, hipMemcpyDeviceToHost, c->last_stream));
    TT2_HIP(hipStreamSynchronize(c->last_stream));
  });
}

tt2_status tt2_train_set_teacher_forcing(tt2_train_ctx* c, const uint8_t* feed_target, int T_out) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    if (!feed_target) {
      c->feed.clear();
      return;
    }
    TT2_CHECK(T_out >= 1 && T_out <= c->Tm, TT2_ERR_SHAPE_MISMATCH, "T_out out of [1, max_T_out]");
    c->feed.assign(feed_target, feed_target + T_out);
  });
}

tt2_status tt2_train_create(const tt2_train_config* cfg, int hip_device, tt2_train_ctx** out) {
  return guard([&] {
    TT2_CHECK(cfg && out, TT2_ERR_INVALID_ARG, "tt2_train_create: null argument");
    *out = nullptr;
    TT2_CHECK(cfg->batch >= 1 && cfg->max_T_in >= 1 && cfg->max_T_out >= 1, TT2_ERR_INVALID_ARG, "bad capacity");
    TT2_CHECK(cfg->max_T_in <= TR_MAX_TIN, TT2_ERR_INVALID_ARG, "max_T_in exceeds the attention kernels' LDS budget");
    TT2_CHECK(cfg->attention_dim >= 1 && cfg->attention_dim <= 256 && 256 % cfg->attention_dim == 0,
              TT2_ERR_INVALID_ARG, "attention_dim must divide 256");
    TT2_CHECK(cfg->attention_filters >= 1 && cfg->attention_filters <= 32, TT2_ERR_INVALID_ARG,
              "attention_filters must be <= 32");
    // LDS tiles of the attention kernels: location-conv window (TR_JT + 64), d context (1024)
    TT2_CHECK(cfg->attention_kernel >= 1 && cfg->attention_kernel <= 65, TT2_ERR_INVALID_ARG,
              "attention_kernel must be <= 65");
    TT2_CHECK(cfg->memory_dim >= 1 && cfg->memory_dim <= 1024, TT2_ERR_INVALID_ARG, "memory_dim must be <= 1024");
    TT2_CHECK(cfg->prenet_units >= 1 && cfg->decoder_lstm_units >= 1 && cfg->num_mels >= 1, TT2_ERR_INVALID_ARG,
              "bad widths");
    int n = 0;
    TT2_HIP(hipGetDeviceCount(&n));
    TT2_CHECK(hip_device >= 0 && hip_device < n, TT2_ERR_HIP, "no such HIP device");
    TT2_HIP(hipSetDevice(hip_device));
    auto* c = new tt2_train_ctx();
    if (const char* e = std::getenv("TT2_TRAIN_BLAS")) c->blas_on = std::atoi(e) != 0;
    if (const char* e = std::getenv("TT2_TR_VALUES16")) c->values16_on = std::atoi(e) != 0;
    if (const char* e = std::getenv("TT2_FE_CONV_DIRECT")) c->fe_direct = std::atoi(e) != 0;
    if (const char* e = std::getenv("TT2_FE_GRU_SEQ")) c->fe_gru_seq = std::atoi(e) != 0;
    {
      const char* e = std::getenv("TT2_TR_PERSIST");
      c->tp_on = !(e && e[0] == '0') && tp_device_ok(hip_device);
      // TT2_TR_PERSIST_BWD=0 runs the per-step backward launches instead of the persistent backward
      const char* eb = std::getenv("TT2_TR_PERSIST_BWD");
      c->tb_on = !(eb && eb[0] == '0') && tb_device_ok(hip_device);
    }
    try {
      c->dev = hip_device;
      c->cfg = *cfg;
      c->B = cfg->batch; c->Tm = cfg->max_T_out; c->Tin = cfg->max_T_in; c->D = cfg->memory_dim;
      c->NM = cfg->num_mels; c->P = cfg->prenet_units; c->H = cfg->decoder_lstm_units; c->A = cfg->attention_dim;
      c->F = cfg->attention_filters; c->KW = cfg->attention_kernel; c->LX1 = c->P + c->D + c->H;
      c->R = cfg->outputs_per_step;
      TT2_CHECK(c->R >= 1 && c->R <= c->Tm, TT2_ERR_INVALID_ARG, "outputs_per_step out of [1, max_T_out]");
      c->PL = cfg->postnet_layers; c->PC = cfg->postnet_channels; c->PK = cfg->postnet_kernel;
      TT2_CHECK(!cfg->postnet || (c->PL >= 1 && c->PL <= 8 && c->PC >= 1 && c->PK >= 1 && c->PK <= 64),
                TT2_ERR_INVALID_ARG,
                "bad postnet shape");
      if (cfg->frontend) {
        c->f_nref = cfg->emt_only ? 1 : 2;
        c->f_adain = cfg->adain != 0;
        TT2_CHECK(cfg->n_emt >= 0 && cfg->n_spk >= 0 && cfg->orthog_weight >= 0.f, TT2_ERR_INVALID_ARG,
                  "n_emt / n_spk / orthog_weight must be >= 0");
        // tacotron.py:68-69; the AdaIN graph builds no style classifiers / orthogonality loss (:485-495, :841)
        TT2_CHECK(!c->f_adain || !cfg->emt_only, TT2_ERR_INVALID_ARG, "must provide speaker reference to use AdaIn");
        TT2_CHECK(!c->f_adain || (cfg->n_emt == 0 && cfg->n_spk == 0 && cfg->orthog_weight == 0.f), TT2_ERR_INVALID_ARG,
                  "adain: no style-embedding classifiers or orthogonality loss (n_emt = n_spk = 0, orthog_weight = 0)");
        int W = cfg->num_mels;
        for (int i = 0; i < 6; ++i) W = (c->f_adain && i >= 2) ? W : (W + 1) / 2;
        c->f_gin = W * cfg->reference_filters[5];
        const int tokd = cfg->num_heads > 0 ? cfg->style_embed_depth / cfg->num_heads : 0;
        const int sw = cfg->use_gst && !c->f_adain ? cfg->num_heads * tokd : 128;  // style embedding width
        TT2_CHECK(cfg->memory_dim == 2 * cfg->encoder_lstm_units + (c->f_adain ? 1 : c->f_nref) * sw, TT2_ERR_INVALID_ARG,
                  c->f_adain    ? "adain: memory_dim must be 2*encoder_lstm_units + 128"
                  : cfg->use_gst ? "memory_dim must be 2*encoder_lstm_units + (emt_only ? 1 : 2) * style_embed_depth"
                                 : "use_gst = 0: memory_dim must be 2*encoder_lstm_units + (emt_only ? 1 : 2) * 128");
        TT2_CHECK(cfg->enc_conv_layers >= 1 && cfg->enc_conv_layers <= 8 && cfg->enc_conv_channels <= 512 &&
                      cfg->n_symbols >= 1 && cfg->embedding_dim >= 1 && cfg->max_T_ref >= 1,
                  TT2_ERR_INVALID_ARG, "bad front-end shape");
        TT2_CHECK(cfg->style_att_dim <= 128 && cfg->num_gst <= 16 && tokd <= 64 && cfg->num_heads >= 1 &&
                      cfg->style_att_dim % cfg->num_heads == 0 && cfg->style_att_dim / cfg->num_heads <= 32 &&
                      cfg->num_heads * cfg->num_gst <= 64,
                  TT2_ERR_INVALID_ARG, "GST shape outside the fe_gst kernels' LDS tiles");
        for (int i = 0; i < 6; ++i)
          TT2_CHECK(cfg->reference_filters[i] >= 1 && cfg->reference_filters[i] <= 512, TT2_ERR_INVALID_ARG,
                    "reference_filters must be in [1, 512]");
      }
      TT2_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      TT2_HIP(hipEventCreate(&c->ev0));
      TT2_HIP(hipEventCreate(&c->ev1));
      tr_build_vars(c);
      tr_alloc(c);

    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

void tt2_train_destroy(tt2_train_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->tp_ctl_host) (void)hipHostFree(c->tp_ctl_host);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

tt2_status tt2_train_load_tensor(tt2_train_ctx* c, const char* name, const float* host, const int64_t* shape, int ndim) {
  return guard([&] {
    TT2_CHECK(c && name && host && (shape || ndim == 0), TT2_ERR_INVALID_ARG, "tt2_train_load_tensor: null argument");
    auto it = c->index.find(name);
    if (it == c->index.end()) return;  // not a decoder-slice variable: ignored (full checkpoints load as-is)
    const TrVar& v = c->vars[it->second];
    long n = 1;
    for (int i = 0; i < ndim; ++i) n *= shape[i];
    TT2_CHECK(n == v.n, TT2_ERR_SHAPE_MISMATCH, std::string("shape mismatch for ") + name);
    TT2_HIP(hipSetDevice(c->dev));
    TT2_HIP(hipMemcpy(c->params.as<float>() + v.off, host, sizeof(float) * n, hipMemcpyHostToDevice));
    c->host[name].shape.assign(shape, shape + ndim);
  });
}

tt2_status tt2_train_finalize(tt2_train_ctx* c) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    for (const auto& v : c->vars)
      TT2_CHECK(c->host.count(v.name), TT2_ERR_NOT_LOADED, "missing variable " + v.name);
    TT2_HIP(hipSetDevice(c->dev));
    TT2_HIP(hipMemset(c->adam_m.p, 0, c->adam_m.bytes));
    TT2_HIP(hipMemset(c->adam_v.p, 0, c->adam_v.bytes));
    c->finalized = true;
  });
}

tt2_status tt2_train_bind_grads_dev(tt2_train_ctx* c, float* grads_d, int64_t* n_out) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    if (n_out) *n_out = c->total + 1;  // the gradients + the step's status word (k_tr_status)
    c->grads = grads_d ? grads_d : c->grads_own.as<float>();
  });
}

tt2_status tt2_train_moving_stats_dev(tt2_train_ctx* c, float* buf_d, int64_t* n_out, int unpack, void* stream) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_train_finalize not called");
    auto is_stat = [](const std::string& n) {
      auto ends = [&](const char* s) {
        const size_t k = std::strlen(s);
        return n.size() >= k && n.compare(n.size() - k, k, s) == 0;
      };
      return ends("moving_mean") || ends("moving_variance");
    };
    int64_t total = 0;
    for (const auto& v : c->vars)
      if (is_stat(v.name)) total += v.n;
    if (n_out) *n_out = total;
    if (!buf_d) return;
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    int64_t o = 0;
    for (const auto& v : c->vars) {
      if (!is_stat(v.name)) continue;
      float* p = c->params.as<float>() + v.off;
      if (unpack)
        TT2_HIP(hipMemcpyAsync(p, buf_d + o, v.n * sizeof(float), hipMemcpyDeviceToDevice, s));
      else
        TT2_HIP(hipMemcpyAsync(buf_d + o, p, v.n * sizeof(float), hipMemcpyDeviceToDevice, s));
      o += v.n;
    }
  });
}

tt2_status tt2_train_forward_backward_dev(tt2_train_ctx* c, const float* memory_d, const int32_t* lengths_d,
                                          const float* targets_d, const float* stop_targets_d,
                                          const uint8_t* prenet_masks_d, const uint8_t* zoneout_masks_d,
                                          const uint8_t* postnet_masks_d, int T_in, int T_out, void* stream) {
  return guard([&] {
    TT2_CHECK(c && memory_d && lengths_d && targets_d && stop_targets_d && prenet_masks_d, TT2_ERR_INVALID_ARG,
              "tt2_train_forward_backward_dev: null argument");
    TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_train_finalize not called");
    TT2_CHECK(T_in >= 1 && T_in <= c->Tin && T_out >= 1 && T_out <= c->Tm, TT2_ERR_SHAPE_MISMATCH,
              "T_in/T_out exceed capacity");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    c->last_stream = s;
    TT2_HIP(hipEventRecord(c->ev0, s));
    TT2_CHECK(!c->cfg.frontend, TT2_ERR_STATE,
              "front-end context: use tt2_train_forward_backward_text_dev (ids + reference mels)");
    tr_forward_backward(c, memory_d, lengths_d, targets_d, stop_targets_d, prenet_masks_d, zoneout_masks_d,
                        postnet_masks_d, T_in, T_out, s);
    tr_redzones(c, "decoder + postnet");
    tr_regularize(c, s);
    tr_write_status(c, s);
    TT2_HIP(hipEventRecord(c->ev1, s));
    TT2_HIP(hipGetLastError());
  });
}

tt2_status tt2_train_forward_backward_text_dev(tt2_train_ctx* c, const int32_t* ids_d, const int32_t* lengths_d,
                                               const float* ref_emt_d, const float* ref_spk_d, int T_ref,
                                               const float* targets_d, const float* stop_targets_d,
                                               const uint8_t* prenet_masks_d, const uint8_t* zoneout_masks_d,
                                               const uint8_t* postnet_masks_d, const uint8_t* enc_conv_masks_d,
                                               const uint8_t* enc_zoneout_masks_d, int T_in, int T_out, void* stream) {
  return guard([&] {
    TT2_CHECK(c && ids_d && lengths_d && ref_emt_d && targets_d && stop_targets_d && prenet_masks_d,
              TT2_ERR_INVALID_ARG, "tt2_train_forward_backward_text_dev: null argument");
    TT2_CHECK(c->cfg.frontend, TT2_ERR_STATE, "context built without cfg.frontend");
    TT2_CHECK(c->f_nref == 1 || ref_spk_d, TT2_ERR_INVALID_ARG, "ref_spk required unless emt_only");
    TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_train_finalize not called");
    TT2_CHECK(T_in >= 1 && T_in <= c->Tin && T_out >= 1 && T_out <= c->Tm, TT2_ERR_SHAPE_MISMATCH,
              "T_in/T_out exceed capacity");
    TT2_CHECK(T_ref >= 1 && T_ref <= c->cfg.max_T_ref, TT2_ERR_SHAPE_MISMATCH, "T_ref exceeds capacity");
    TT2_CHECK(!(c->cfg.n_emt > 0 || (c->f_nref == 2 && c->cfg.n_spk > 0)) || c->has_labels, TT2_ERR_STATE,
              "style-embedding classifiers (n_emt / n_spk > 0) need tt2_train_set_style_labels first");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    c->last_stream = s;
    TT2_HIP(hipEventRecord(c->ev0, s));
    const float* refs[2] = {ref_emt_d, ref_spk_d};
    g_tr_kpart = &c->kpart;
    g_tr_prec = c->cfg.precision ? 2 : 0;
    g_tr_ctx = c;
    tr_front_forward(c, ids_d, lengths_d, refs, T_ref, enc_conv_masks_d, enc_zoneout_masks_d, T_in, s);
    tr_redzones(c, "front forward");
    tr_forward_backward(c, c->fMEM.as<float>(), lengths_d, targets_d, stop_targets_d, prenet_masks_d, zoneout_masks_d,
                        postnet_masks_d, T_in, T_out, s);
    tr_redzones(c, "decoder + postnet");
    g_tr_kpart = &c->kpart;
    g_tr_prec = c->cfg.precision ? 2 : 0;
    g_tr_ctx = c;
    tr_front_backward(c, ids_d, lengths_d, refs, T_ref, enc_conv_masks_d, enc_zoneout_masks_d, T_in, s);
    tr_redzones(c, "front backward");
    g_tr_kpart = nullptr;
    g_tr_prec = 0;
    g_tr_ctx = nullptr;
    tr_regularize(c, s);
    tr_write_status(c, s);
    TT2_HIP(hipEventRecord(c->ev1, s));
    TT2_HIP(hipGetLastError());
  });
}

tt2_status tt2_train_apply_dev(tt2_train_ctx* c, float lr, int global_step, void* stream) {
  return guard([&] {
    TT2_CHECK(c && c->finalized, TT2_ERR_NOT_LOADED, "tt2_train_apply_dev: not finalized");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    c->last_stream = s;
    tr_apply(c, lr, global_step, s);
    tr_redzones(c, "apply");
    TT2_HIP(hipGetLastError());
  });
}

tt2_status tt2_train_losses(tt2_train_ctx* c, float* out4 /* [5] */, float* fb_ms) {
  return guard([&] {
    TT2_CHECK(c && out4, TT2_ERR_INVALID_ARG, "null argument");
    TT2_HIP(hipSetDevice(c->dev));
    // read back in the order of the stream that produced the values: a synchronous hipMemcpy of a
    // few bytes after hipDeviceSynchronize() returned stale data here (small D2H copies are served
    // by the host through the BAR and missed the last kernels' L2-resident writes)
    TT2_HIP(hipMemcpyAsync(out4, c->red.p, sizeof(float) * 5, hipMemcpyDeviceToHost, c->last_stream));
    TT2_HIP(hipStreamSynchronize(c->last_stream));
    tr_persist_check(c);
    if (!c->cfg.postnet) out4[4] = 0.f;
    if (fb_ms) TT2_HIP(hipEventElapsedTime(fb_ms, c->ev0, c->ev1));
  });
}

tt2_status tt2_train_get_tensor(tt2_train_ctx* c, const char* name, int which, float* host) {
  return guard([&] {
    TT2_CHECK(c && name && host, TT2_ERR_INVALID_ARG, "null argument");
    TT2_HIP(hipSetDevice(c->dev));
    TT2_HIP(hipDeviceSynchronize());
    tr_persist_check(c);
    if (std::string(name) == "diag:blas_calls") {  // gemm_bf16_kc products issued since create (1 float)
      host[0] = (float)c->blas_calls;
      return;
    }
    if (std::string(name) == "diag:persist") {  // 1 when the last forward ran the persistent launch
      host[0] = c->tp_last ? 1.f : 0.f;
      return;
    }
    if (std::string(name) == "diag:persist_bwd") {  // 1 when the last backward ran the persistent launch
      host[0] = c->tb_last ? 1.f : 0.f;
      return;
    }
    if (std::string(name) == "memory") {  // d loss / d memory of the last forward_backward
      tr_d2h(c, host, c->DMEM.p, sizeof(float) * (size_t)c->B * c->Tin_last * c->D);
      return;
    }
    if (c->cfg.postnet && std::string(name) == "postnet:projection") {  // Postnet residual [B,T,NM]
      tr_d2h(c, host, c->PPRJ.p, sizeof(float) * (size_t)c->B * c->Tf_last * c->NM);
      return;
    }
    if (c->cfg.frontend && std::string(name) == "frontend:memory") {  // the front end's memory [B,T_in,D]
      tr_d2h(c, host, c->fMEM.p, sizeof(float) * (size_t)c->B * c->Tin_last * c->D);
      return;
    }
    if (c->cfg.frontend && std::string(name).rfind("debug:", 0) == 0) {
      // the encoder conv-1 backward operands as the last text step left them: the embedding output
      // [B*T_in][E], its transposed im2col [K*E][B*T_in] and conv-1's dz [B*T_in][C]
      const long M = (long)c->B * c->Tin_last, E = c->cfg.embedding_dim, C = c->cfg.enc_conv_channels;
      const std::string n(name);
      if (n == "debug:enc_embedded") tr_d2h(c, host, c->fEX.p, sizeof(float) * (size_t)(M * E));
      else if (n == "debug:enc_conv1_im2col") tr_d2h(c, host, c->fFBUF.p, sizeof(float) * (size_t)(c->cfg.enc_conv_kernel * E * M));
      else if (n == "debug:enc_conv1_dz") tr_d2h(c, host, c->fDZc.p, sizeof(float) * (size_t)(M * C));
      else TT2_CHECK(false, TT2_ERR_INVALID_ARG, "unknown debug tensor " + n);
      return;
    }
    for (int r = 0; r < c->f_nref; ++r)  // reference embeddings (ReferenceEncoder outputs) [B,128]
      if (std::string(name) == (r == 0 ? "frontend:refnet_emt" : "frontend:refnet_spk")) {
        tr_d2h(c, host, c->fREF[r].p, sizeof(float) * (size_t)c->B * 128);
        return;
      }
    auto it = c->index.find(name);
    TT2_CHECK(it != c->index.end(), TT2_ERR_INVALID_ARG, std::string("unknown variable ") + name);
    const TrVar& v = c->vars[it->second];
    const float* base = which == 0 ? c->params.as<float>() : which == 1 ? c->grads
                      : which == 2 ? c->adam_m.as<float>() : c->adam_v.as<float>();
    TT2_CHECK(which >= 0 && which <= 3, TT2_ERR_INVALID_ARG, "which must be 0..3");
    tr_d2h(c, host, base + v.off, sizeof(float) * v.n);
  });
}

tt2_status tt2_train_outputs(tt2_train_ctx* c, float* frames, float* stop_logits, float* alignments) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    TT2_HIP(hipSetDevice(c->dev));
    TT2_HIP(hipDeviceSynchronize());
    const int B = c->B, T = c->T_last, R = c->R, Tf = c->Tf_last, NM = c->NM, Tin = c->Tin_last;
    // device layouts are step-major [T][B][r·..]; the ABI returns frames [B][T·r][..] like
    // tower_decoder_output (tacotron.py:355-358: reshape [B, -1, num_mels])
    if (frames) {
      std::vector<float> tmp((size_t)Tf * B * NM);
      tr_d2h(c, tmp.data(), c->FR.p, sizeof(float) * tmp.size());
      for (int f = 0; f < Tf; ++f)
        for (int b = 0; b < B; ++b)
          std::memcpy(frames + ((size_t)b * Tf + f) * NM, tmp.data() + (((size_t)(f / R) * B + b) * R + f % R) * NM,
                      sizeof(float) * NM);
    }
    if (stop_logits) {
      std::vector<float> tmp((size_t)Tf * B);
      tr_d2h(c, tmp.data(), c->ST.p, sizeof(float) * tmp.size());
      for (int f = 0; f < Tf; ++f)
        for (int b = 0; b < B; ++b) stop_logits[(size_t)b * Tf + f] = tmp[((size_t)(f / R) * B + b) * R + f % R];
    }
    if (alignments)  // [B][Tin][T] already
      tr_d2h(c, alignments, c->ALIGN.p, sizeof(float) * (size_t)B * Tin * T);
  });
}

}  // extern "C"
