// Persistent teacher-forced decoder forward of the training step (train_persist.h).
//
// Why: at B = 64 the per-step products of the launch loop (k_tr_fused x2, the query GEMM, the
// energy and context kernels: 5 launches per decoder step) run at 7-13 us each although each is
// ~1 us of MFMA / HBM work: the bf16 LSTM weights (35 MB) are re-streamed from the MALL every step
// and every launch pays its ramp.  The chip holds them: 256 work-groups x 136 KB of B fragments
// in VGPRs, so a step only moves activations between work-groups.
//
// Roles of work-group g (all 256 have both):
//   LSTM       hidden units [4g, 4g+4) of both layers = 16 gate columns (gate q, unit u at column
//              4q + u), all 64 (padded) rows; v_mfma_f32_16x16x32_bf16, K split over the 4 waves
//              (one per SIMD, 512 registers per lane: 136 of them hold the weight fragments)
//   attention  row b = g & 63, quarter s = g >> 6: attention dims [32s, 32s+32) (query columns,
//              keys, location projection, energies) and context channels [256s, 256s+256); the 4
//              quarters of a row have equal g % 8 (one XCD under round-robin placement: speed only)
//
// LSTM-1 gates = prenet_t·W1p + hz1_{t-1}·W1h + ctx_{t-1}·W1c: the first two terms are off the
// recurrence's chain (computed during step t-1's attention), only ctx·W1c waits for the context.
// LSTM-2 gates = hz2_{t-1}·W2h (off the chain, computed after the previous context) + h1_t·W2i.
//
// One step t (tag t+1, exchange buffers by parity t & 1):
//   L1   wave w waits CTX(t-1) of quarter w (its 256 context k), ctx·W1c, + off-chain terms ->
//        cell + zoneout (k_tr_fused<TF_FWD>'s epilogue) -> h1, hz1 (bf16, A-fragment layout) -> H1
//   L2   wave w waits H1 of producers [64w, 64w+64) (its 256 k), h1·W2i + off-chain -> cell ->
//        h2, hz2 -> H2
//   ATT  wait H2 (all; wave w polls lines 2w, 2w+1), h2 row -> query quarter (bf16 operands, fp32 sums),
//        location features, energy partials over this quarter's 32 dims -> granules to the other
//        3 quarters; off-chain L1 terms of t+1 (prenet_{t+1}·W1p + hz1_t·W1h); take the partials
//        (summed in quarter order: identical in all four), masked softmax, cumulative alignments,
//        context quarter -> CTX; off-chain L2 terms of t+1 (hz2_t·W2h)
// Every exchanged byte is an sc1 (write-through) store, drained by every wave before one barrier and
// the flag stores (8 replicas per line, consumer XCD group g % 8 polls its own); every read of it is
// an sc1 load by a wave that polled the producers' flags itself or joined a barrier behind such a
// poll (MI355X_MICROARCH.md § visibility, Valid forms row 1).  Energy partials are data-tagged 8-byte
// granules (Guideline 16 R2).  The plain activation-slot stores are consumed only after the launch.
// Spins are bounded (2 s on s_memrealtime); a timeout or a peer's failure ends every work-group and
// the host reports the phase.
#include "tp_device.h"

// 1: every LSTM weight fragment of the work-group's 16 gate columns register-resident (the off-chain
// rows too: 72 more registers per lane); 0: the off-chain rows streamed from L2 / MALL each step
#ifndef TP_RESIDENT_OFFCHAIN
#define TP_RESIDENT_OFFCHAIN 1
#endif

namespace tt2 {

enum { TP_PH_H1 = 0, TP_PH_H2 = 1, TP_PH_CTX = 2, TP_PH_E = 3 };
constexpr int TP_NW = TP_NT / 64;          // waves
constexpr int TP_KSW = 32 / TP_NW;         // k-steps per wave of a 1024-deep segment
constexpr int TP_PKW = TP_P / 32 / TP_NW;  // prenet k-steps per wave
constexpr int TP_RG = TP_NT / 32;          // attention row groups (32 dims each)
constexpr int TP_VG = TP_NT / 128;         // context row groups (128 channel pairs each)
static_assert(TP_KSW % 4 == 0 && TP_PKW >= 1 && TP_H == 1024 && TP_D == 1024, "train_persist geometry");

// LDS layout (floats)
constexpr int TP_KW = 31;                       // attention_kernel (fork default; tr_persist_fits)
constexpr int TPL_RED = 0;                      // [TP_NW waves][64][16] partial gate tiles
constexpr int TPL_WQ = TPL_RED + TP_NW * 1024;  // query columns of this quarter as bf16 B fragments
constexpr int TPL_CW = TPL_WQ + TP_H * 32 / 2;  // [15 + TMAX + 17 + 16] cumulative alignments, zero padded
constexpr int TPL_QP = TPL_CW + TP_TMAX + 48;   // [TP_NW][32] query partials
constexpr int TPL_QV = TPL_QP + TP_NW * 32;     // [32] q + b_a
constexpr int TPL_EP = TPL_QV + 32;             // [TMAX] this quarter's energy partials
constexpr int TPL_AL = TPL_EP + TP_TMAX;        // [TMAX] energies -> alignments (zero past T_in)
constexpr int TPL_CR = TPL_AL + TP_TMAX;        // [TP_VG][256] context partials
constexpr int TPL_SC = TPL_CR + TP_VG * 256;    // [16] reduction scratch, then ints
constexpr int TPL_END = TPL_SC + 32;
static_assert(TP_TMAX % 64 == 0 && TP_TMAX <= TP_NT && TP_VG == 2, "train_persist attention geometry");

size_t tp_lds_bytes() { return sizeof(float) * (size_t)TPL_END; }

// constant address space: uniform reads of kernel-lifetime constants become scalar (s_load) reads
typedef const __attribute__((address_space(4))) float tp_cf;
__device__ __forceinline__ tp_cf* tp_const(const float* p) { return (tp_cf*)(p); }

// wave partial tiles (4 row tiles x 16 columns) -> red[w][64][16]
__device__ __forceinline__ void tp_put_tiles(float* red, const tp_f4 (&acc)[4], int w, int lane) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w * 1024 + (16 * mt + 4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[mt][r];
}

// acc[mt] += X[rows of tile mt][k-steps ks0 .. ks0 + N) · W (B fragments wf[0..N)), X a [64][K]
// A-fragment-layout bf16 buffer: one per-lane offset, the (tile, k-step) block offset in the
// uniform soffset (ks0 wave-uniform), every load of the batch in flight at once; sc1 loads for
// exchanged rows
template <int N, bool SC1>
__device__ __forceinline__ void tp_mfma_rows(tp_f4 (&acc)[4], const __bf16* X, int K, int ks0, const tp_bf8 (&wf)[N],
                                             int lane) {
  const auto rs = tp_rsrc(X);
  const int vo = ((lane & 15) * 32 + 8 * (lane >> 4)) * 2;
  tp_bf8 af[N * 4];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) af[i * 4 + mt] = tp_ldx4<SC1>(rs, vo, (mt * (K >> 5) + ks0 + i) * 1024);
  tp_wait(af);
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i * 4 + mt], wf[i], acc[mt], 0, 0, 0);
}

// the same with the B fragments streamed from the bf16 W^T row of this lane's column (wvo: the
// lane's byte offset of its column row + 8 (lane >> 4) k; k-step ks0 + i at k = wk0 + 32 i): the
// off-chain products, whose weights stay in L2 / MALL
template <int N, bool SC1>
__device__ __forceinline__ void tp_mfma_stream(tp_f4 (&acc)[4], const __bf16* X, int K, int ks0, const __bf16* Wt,
                                               int wvo, int wk0, int lane) {
  const auto rs = tp_rsrc(X), rw = tp_rsrc(Wt);
  const int vo = ((lane & 15) * 32 + 8 * (lane >> 4)) * 2;
  tp_bf8 f[N * 5];  // [0, 4N): A fragments, [4N, 5N): B fragments
#pragma unroll
  for (int i = 0; i < N; ++i) f[4 * N + i] = tp_ldx4<false>(rw, wvo, (wk0 + 32 * i) * 2);
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) f[i * 4 + mt] = tp_ldx4<SC1>(rs, vo, (mt * (K >> 5) + ks0 + i) * 1024);
  tp_wait(f);
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[i * 4 + mt], f[4 * N + i], acc[mt], 0, 0, 0);
}

// a wave's TP_KSW k-steps of exchanged rows, loaded four at a time (register budget)
__device__ __forceinline__ void tp_mfma_seg(tp_f4 (&acc)[4], const __bf16* X, int K, int ks0,
                                            const tp_bf8 (&wf)[TP_KSW], int lane) {
#pragma unroll
  for (int c = 0; c < TP_KSW; c += 4) {
    const tp_bf8 part[4] = {wf[c], wf[c + 1], wf[c + 2], wf[c + 3]};
    tp_mfma_rows<4, true>(acc, X, K, ks0 + c, part, lane);
  }
}

__device__ __forceinline__ float tp_block_max(float v, float* scr) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scr[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = scr[0];
#pragma unroll
  for (int i = 1; i < TP_NW; ++i) r = fmaxf(r, scr[i]);
  return r;
}
__device__ __forceinline__ float tp_block_sum(float v, float* scr) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scr[8 + (threadIdx.x >> 6)] = v;
  __syncthreads();
  float r = scr[8];
#pragma unroll
  for (int i = 1; i < TP_NW; ++i) r += scr[8 + i];
  return r;
}

__global__ __launch_bounds__(TP_NT, 1) void k_tr_persist(TpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const red = sm + TPL_RED;
  tp_bf8* const wqf = reinterpret_cast<tp_bf8*>(sm + TPL_WQ);
  float* const cw = sm + TPL_CW;
  float* const qps = sm + TPL_QP;
  float* const qv = sm + TPL_QV;
  float* const ep = sm + TPL_EP;
  float* const al = sm + TPL_AL;
  float* const cr = sm + TPL_CR;
  float* const scr = sm + TPL_SC;
  int* const sfail = reinterpret_cast<int*>(sm + TPL_SC + 16);
  constexpr int H = TP_H, P = TP_P, D = TP_D, A = TP_A, LX1 = TP_LX1, TM = TP_TMAX;
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: offsets live in SGPRs
  const int B = a.B, T = a.T, Tin = a.Tin;
  const int rb = g & 63, sib = g >> 6;  // attention row, quarter
  const bool arow = rb < B;

  // ---- resident LSTM weights: B fragments of gate columns (lane & 15) -> gate n >> 2, unit 4g + (n & 3)
  const int fn = lane & 15, fk = 8 * (lane >> 4);
  // chain weights (context rows of W1, h1 rows of W2) resident; the off-chain rows (prenet, zoned
  // h) are streamed by the off-chain products from L2 / MALL
  tp_bf8 w1c[TP_KSW], w2i[TP_KSW];
#if TP_RESIDENT_OFFCHAIN
  tp_bf8 w1h[TP_KSW], w2h[TP_KSW], w1p[TP_PKW];  // the off-chain rows too (zoned h of both layers, prenet)
#endif
  const int wcol = (fn >> 2) * H + 4 * g + (fn & 3);
  const int wvo1 = (wcol * LX1 + fk) * 2, wvo2 = (wcol * 2 * H + fk) * 2;  // bytes (K1T / K2T < 2 GB)
  const int wk0 = 32 * TP_KSW * w;
#pragma unroll
  for (int i = 0; i < TP_KSW; ++i) {
    w1c[i] = *reinterpret_cast<const tp_bf8*>(a.K1T + (long)wcol * LX1 + P + wk0 + 32 * i + fk);
    w2i[i] = *reinterpret_cast<const tp_bf8*>(a.K2T + (long)wcol * 2 * H + wk0 + 32 * i + fk);
#if TP_RESIDENT_OFFCHAIN
    w1h[i] = *reinterpret_cast<const tp_bf8*>(a.K1T + (long)wcol * LX1 + P + D + wk0 + 32 * i + fk);
    w2h[i] = *reinterpret_cast<const tp_bf8*>(a.K2T + (long)wcol * 2 * H + H + wk0 + 32 * i + fk);
#endif
  }
#if TP_RESIDENT_OFFCHAIN
#pragma unroll
  for (int i = 0; i < TP_PKW; ++i) w1p[i] = *reinterpret_cast<const tp_bf8*>(a.K1T + (long)wcol * LX1 + 32 * TP_PKW * w + 32 * i + fk);
#endif
  // LSTM epilogue thread (tid < 256): row er, unit en = 4g + eu; its cell state lives in registers
  static_assert(TP_NT >= 256, "one epilogue thread per (row, unit)");
  const int er = tid >> 2, eu = tid & 3, en = 4 * g + eu;
  const bool eth = tid < 256, erow = eth && er < B;
  float bias1[4], bias2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bias1[q] = eth ? a.b1[q * H + en] : 0.f;
    bias2[q] = eth ? a.b2[q * H + en] : 0.f;
  }
  float c1 = 0.f, hz1 = 0.f, c2 = 0.f, hz2 = 0.f;
  const int evo = er * H + en;  // (row, unit) element offset in the [B][H] planes

  // ---- attention row constants.  Energies as v_mfma_f32_16x16x4f32 tiles of U^T = KW^T·C^T (dims x
  // positions, C the cum Toeplitz): wave w owns the position tiles nt = w + 4r, lane l the position
  // 16 nt + (l & 15) and the dims 16 mt + 4 (l >> 4) + i of both dim tiles mt.  Context: channel pair
  // vcp, positions [TM/2 vg, TM/2 vg + TM/2)
  const int vcp = tid & 127, vg = tid >> 7;
  const int jl = lane & 15, g4 = lane >> 4;
  constexpr int NTW = TM / 16 / TP_NW;  // position tiles per wave
  float key[NTW * 8];     // AGPRs: keys[rb][16 (w + 4 r) + jl][32 sib + 16 mt + 4 g4 + i] at [8 r + 4 mt + i]
  float vals[TM / 2];     // AGPRs: bf16 pairs of values16[rb][TM/2 vg + i][256 sib + 2 vcp]
  float kwa[16];          // A fragments: KW^T[32 sib + 16 mt + jl][4 ks + g4] at [8 mt + ks] (tap 31 -> 0)
  float vav[8];           // v_a of the lane's dims [4 mt + i]
#pragma unroll
  for (int r = 0; r < NTW; ++r) {
    const int j = 16 * (w + 4 * r) + jl;
    const bool kj = arow && j < Tin;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const tp_f4 v = kj ? *reinterpret_cast<const tp_f4*>(a.keys + ((long)rb * Tin + j) * A + 32 * sib + 16 * mt + 4 * g4)
                         : tp_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) key[8 * r + 4 * mt + i] = tp_aput(v[i]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      kwa[8 * mt + ks] = (4 * ks + g4 < TP_KW) ? a.KWT[(32 * sib + 16 * mt + jl) * 32 + 4 * ks + g4] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) vav[4 * mt + i] = a.va[32 * sib + 16 * mt + 4 * g4 + i];
  }
#pragma unroll
  for (int i = 0; i < TM / 2; ++i) {
    const int j = (TM / 2) * vg + i;
    const unsigned v = (arow && j < Tin)
                           ? *reinterpret_cast<const unsigned*>(a.values16 + ((long)rb * Tin + j) * D + 256 * sib + 2 * vcp)
                           : 0u;
    vals[i] = tp_aput(__uint_as_float(v));
  }
  // q-side constant of dim tid < 32: b_a + bc·W_loc (the location conv's bias through W_loc)
  const float qbias = (arow && tid < 32) ? a.ba[32 * sib + tid] + a.KWT[(32 * sib + tid) * 32 + 31] : 0.f;
  int len = 0;
  if (arow) {
    len = a.lens[rb];
    // query columns as B fragments: k-step ks, column tile nt, lane l holds
    // Wq[32 ks + 8 (l >> 4) + e][32 sib + 16 nt + (l & 15)], e < 8
    for (int e = tid; e < 32 * 2 * 64; e += TP_NT) {
      const int l = e & 63, nt = (e >> 6) & 1, ks = e >> 7;
      const __bf16* src = a.Wq + (long)(32 * ks + 8 * (l >> 4)) * A + 32 * sib + 16 * nt + (l & 15);
      tp_bf8 v;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = src[(long)k * A];
      wqf[e] = v;
    }
  }
  for (int e = tid; e < TM + 48; e += TP_NT) cw[e] = 0.f;
  for (int e = tid; e < TM; e += TP_NT) al[e] = 0.f;
  if (tid == 0) sfail[0] = 0;

  // ---- off-chain products, accumulated per wave in registers between the chain's waits and added to
  // the wave's chain partial tiles (so the cell's sum over the waves covers both):
  //   ao1 = prenet_{t+1}·W1p (after CTX(t) is published) + hz1_t·W1h (after H2(t) is published)
  //   ao2 = hz2_t·W2h (while the energy partials of step t travel)
  tp_f4 ao1[4] = {}, ao2[4] = {};
#if TP_RESIDENT_OFFCHAIN
  auto prenet_part = [&](int tn) {  // prenet_tn·W1p, k-steps [TP_PKW w, TP_PKW (w + 1)) of the prenet rows
    tp_mfma_rows<TP_PKW, false>(ao1, a.preh + (long)tn * 64 * P, P, TP_PKW * w, w1p, lane);
  };
  // hz·W over k-steps [c0, c1) of this wave's segment (4 at a time: register budget)
  auto hz_seg = [&](tp_f4(&acc)[4], const __bf16* X, const tp_bf8(&wf)[TP_KSW], int c0, int c1) {
#pragma unroll
    for (int c = 0; c < TP_KSW; c += 4) {
      if (c < c0 || c >= c1) continue;
      const tp_bf8 part[4] = {wf[c], wf[c + 1], wf[c + 2], wf[c + 3]};
      tp_mfma_rows<4, true>(acc, X, H, TP_KSW * w + c, part, lane);
    }
  };
  auto hz1_part = [&](int t0, int c0 = 0, int c1 = TP_KSW) {  // hz1_t0·W1h (the producers its L2 wait covered)
    hz_seg(ao1, a.Z1X + (long)(t0 & 1) * 64 * H, w1h, c0, c1);
  };
  auto hz2_part = [&](int t0, int c0 = 0, int c1 = TP_KSW) {  // hz2_t0·W2h (the producers its H2 wait covered)
    hz_seg(ao2, a.Z2X + (long)(t0 & 1) * 64 * H, w2h, c0, c1);
  };
#else
  auto prenet_part = [&](int tn) {  // prenet_tn·W1p, k-steps [TP_PKW w, TP_PKW (w + 1)) of the prenet rows
    tp_mfma_stream<TP_PKW, false>(ao1, a.preh + (long)tn * 64 * P, P, TP_PKW * w, a.K1T, wvo1, 32 * TP_PKW * w, lane);
  };
  auto hz1_part = [&](int t0, int c0 = 0, int c1 = TP_KSW) {  // hz1_t0·W1h (the producers its L2 wait covered)
#pragma unroll
    for (int c = 0; c < TP_KSW; c += 4)
      if (c >= c0 && c < c1)
        tp_mfma_stream<4, true>(ao1, a.Z1X + (long)(t0 & 1) * 64 * H, H, TP_KSW * w + c, a.K1T, wvo1, P + D + wk0 + 32 * c,
                                lane);
  };
  auto hz2_part = [&](int t0, int c0 = 0, int c1 = TP_KSW) {  // hz2_t0·W2h (the producers its H2 wait covered)
#pragma unroll
    for (int c = 0; c < TP_KSW; c += 4)
      if (c >= c0 && c < c1)
        tp_mfma_stream<4, true>(ao2, a.Z2X + (long)(t0 & 1) * 64 * H, H, TP_KSW * w + c, a.K2T, wvo2, H + wk0 + 32 * c,
                                lane);
  };
#endif
  prenet_part(0);  // hz1_{-1} = hz2_{-1} = 0
  __syncthreads();

  // one LSTM layer's epilogue for thread (er, eu): gates = bias + off-chain + Σ wave partials
  // (k_tr_fused<TF_FWD>'s cell + zoneout, Architecture_wrappers.py:214-224 / modules.py:236-244)
  struct Cell {
    float si, tj, sf, so, cn, hn, cz, hz;
  };
  auto cell = [&](const float (&bias)[4], float cp, float hp, float kc, float kh) {
    float pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ci = er * 16 + 4 * q + eu;
      float s = red[ci];
#pragma unroll
      for (int ww = 1; ww < TP_NW; ++ww) s += red[ww * 1024 + ci];
      pre[q] = bias[q] + s;
    }
    Cell o;
    o.si = tp_sigm(pre[0]);
    o.tj = tanhf(pre[1]);
    o.sf = tp_sigm(pre[2] + 1.0f);
    o.so = tp_sigm(pre[3]);
    o.cn = o.sf * cp + o.si * o.tj;
    o.hn = o.so * tanhf(o.cn);
    if (a.zm) {
      o.cz = cp + kc * (o.cn - cp);
      o.hz = hp + kh * (o.hn - hp);
    } else {
      o.cz = (1.f - a.z) * o.cn + a.z * cp;
      o.hz = (1.f - a.z) * o.hn + a.z * hp;
    }
    return o;
  };
  // h / zoned h of the 4 units of row er -> one 8-byte write-through store each (lane eu == 0)
  auto xstore = [&](__bf16* X, float hn, float hz, __bf16* Z, int par) {
    const int src = lane & ~3;
    const float h0 = __shfl(hn, src), h1 = __shfl(hn, src + 1), h2 = __shfl(hn, src + 2), h3 = __shfl(hn, src + 3);
    const float z0 = __shfl(hz, src), z1 = __shfl(hz, src + 1), z2 = __shfl(hz, src + 2), z3 = __shfl(hz, src + 3);
    if (erow && eu == 0) {
      const int off = (int)(((long)par * 64 * H + tp_afl(er, 4 * g, H)) * 2);
      tp_st8(X, off, tp_u2{tp_pack(h0, h1), tp_pack(h2, h3)});
      tp_st8(Z, off, tp_u2{tp_pack(z0, z1), tp_pack(z2, z3)});
    }
  };

  // the backward's packed unit operands of one layer (TpArgs::BPK): quads k4, k4 + 1 of this thread
  auto bpk_store = [&](int t, int k4, const Cell& o, float cp, float kc, float kh) {
    const auto rp = tp_rsrc(a.BPK + ((long)t * TP_NB + g) * 4 * TP_NT * 4);
    __builtin_amdgcn_raw_buffer_store_b128(
        tp_u4{__float_as_uint(o.si), __float_as_uint(o.tj), __float_as_uint(o.sf), __float_as_uint(o.so)}, rp,
        (k4 * TP_NT + tid) * 16, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(
        tp_u4{__float_as_uint(o.cn), __float_as_uint(cp), __float_as_uint(kc), __float_as_uint(kh)}, rp,
        ((k4 + 1) * TP_NT + tid) * 16, 0, 0);
  };
#define TP_STAMP(i)                                                         \
  do {                                                                      \
    if (stp && tid == 0) stp[g * 32 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  for (int t = 0; t < T; ++t) {
    const int par = t & 1;
    const unsigned tag = (unsigned)t + 1u;
    long long* const stp = t == a.stamp_step ? a.stamps : nullptr;
    // compiler barrier: the step's LDS-resident constants (query fragments, conv taps, W_loc columns)
    // are re-read every step instead of being hoisted into registers the LSTM products need
    asm volatile("" ::: "memory");
    TP_STAMP(0);
    // zoneout keep bits of both layers for this thread's (row, unit), loaded ahead of the waits
    float kc1 = 0.f, kh1 = 0.f, kc2 = 0.f, kh2 = 0.f;
    if (erow && a.zm) {
      const auto rz = tp_rsrc(a.zm + (long)t * 4 * B * H);
      const int zs = B * H;
      kc1 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, 0, 0);
      kh1 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, zs, 0);
      kc2 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, 2 * zs, 0);
      kh2 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, 3 * zs, 0);
    }
    // ================= L1: ctx_{t-1}·W1c (wave w: context k of quarter (TP_KSW w) / 8)
    {
      tp_f4 acc[4] = {ao1[0], ao1[1], ao1[2], ao1[3]};
      if (t > 0) {
        if (!tp_poll(a, TP_PH_CTX, 64 * ((TP_KSW * w) >> 3), B, tag - 1u)) sfail[0] = 1;
        TP_STAMP(1);
        tp_mfma_seg(acc, a.CX + (long)((t - 1) & 1) * 64 * D, D, TP_KSW * w, w1c, lane);
      }
      tp_put_tiles(red, acc, w, lane);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) ao1[mt] = tp_f4{0.f, 0.f, 0.f, 0.f};
      TP_STAMP(2);
      __syncthreads();
      TP_STAMP(3);
      if (sfail[0]) return;
      Cell o{};
      if (eth) o = cell(bias1, c1, hz1, kc1, kh1);
      xstore(a.H1X, o.hn, o.hz, a.Z1X, par);
      tp_publish(a, TP_PH_H1, tag);
      TP_STAMP(4);
      if (erow) {  // activation slots of step t (plain buffer stores off uniform per-step bases)
        const long tb = (long)t * B;
        const float* g1 = a.G1 + tb * 4 * H;
        const int go = (er * 4 * H + en) * 4;
        tp_bst(g1, go, 0, o.si);
        tp_bst(g1, go, H * 4, o.tj);
        tp_bst(g1, go, 2 * H * 4, o.sf);
        tp_bst(g1, go, 3 * H * 4, o.so);
        tp_bst(a.CN1 + tb * H, evo * 4, 0, o.cn);
        tp_bst(a.C1 + (tb + B) * H, evo * 4, 0, o.cz);
        tp_bst(a.X2 + tb * 2 * H, (er * 2 * H + en) * 4, 0, o.hn);
        tp_bst(a.X1 + (tb + B) * LX1, (er * LX1 + P + D + en) * 4, 0, o.hz);
        if (a.BPK) bpk_store(t, 2, o, c1, a.zm ? kc1 : 1.f - a.z, a.zm ? kh1 : 1.f - a.z);
        c1 = o.cz;
        hz1 = o.hz;
      }
    }
    // ================= L2: h1_t·W2i (wave w: k-steps [TP_KSW w, TP_KSW (w+1)) = producers [8 TP_KSW w, ..))
    {
      tp_f4 acc[4] = {ao2[0], ao2[1], ao2[2], ao2[3]};
      if (!tp_poll(a, TP_PH_H1, 8 * TP_KSW * w, 8 * TP_KSW, tag)) sfail[0] = 1;
      TP_STAMP(5);
      tp_mfma_seg(acc, a.H1X + (long)par * 64 * H, H, TP_KSW * w, w2i, lane);
      tp_put_tiles(red, acc, w, lane);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) ao2[mt] = tp_f4{0.f, 0.f, 0.f, 0.f};
      TP_STAMP(6);
      __syncthreads();
      if (sfail[0]) return;
      Cell o{};
      if (eth) o = cell(bias2, c2, hz2, kc2, kh2);
      xstore(a.H2X, o.hn, o.hz, a.Z2X, par);
      tp_publish(a, TP_PH_H2, tag);
      TP_STAMP(7);
      if (erow) {
        const long tb = (long)t * B;
        const float* g2 = a.G2 + tb * 4 * H;
        const int go = (er * 4 * H + en) * 4;
        tp_bst(g2, go, 0, o.si);
        tp_bst(g2, go, H * 4, o.tj);
        tp_bst(g2, go, 2 * H * 4, o.sf);
        tp_bst(g2, go, 3 * H * 4, o.so);
        tp_bst(a.CN2 + tb * H, evo * 4, 0, o.cn);
        tp_bst(a.C2 + (tb + B) * H, evo * 4, 0, o.cz);
        tp_bst(a.PIN + tb * (H + D), (er * (H + D) + en) * 4, 0, o.hn);
        tp_bst(a.X2 + (tb + B) * 2 * H, (er * 2 * H + H + en) * 4, 0, o.hz);
        if (a.BPK) bpk_store(t, 0, o, c2, a.zm ? kc2 : 1.f - a.z, a.zm ? kh2 : 1.f - a.z);
        c2 = o.cz;
        hz2 = o.hz;
      }
    }
    const bool more = t + 1 < T;
    // Off-chain products of step t+1 in the chain's three hand-off windows (H2, E, CTX): every one of
    // them re-reads a 128 KB exchange buffer in each of the 256 work-groups (32 MB of MALL traffic per
    // product and step), so where they sit moves the chain's own loads.  oc_mode 0:
    // hz1_t·W1h in the H2 window, hz2_t·W2h in the E window, prenet_{t+1}·W1p in the CTX window;
    // 1: hz1 split over the H2 and E windows, hz2 + prenet in the CTX window; 2: as 1 with the
    // prenet term in the H2 window; 3: as 1 with hz2's first half in the E window
    const int ocm = a.oc_mode;
    if (more) {
      if (ocm == 0) {
        hz1_part(t);
      } else {
        hz1_part(t, 0, TP_KSW / 2);
        if (ocm == 2) prenet_part(t + 1);
      }
    }
    TP_STAMP(9);
    // ================= H2 of every producer (wave w polls its 8 TP_KSW producers), then the attention row
    if (!tp_poll(a, TP_PH_H2, 8 * TP_KSW * w, 8 * TP_KSW, tag)) sfail[0] = 1;
    __syncthreads();
    TP_STAMP(8);
    if (sfail[0]) return;
    if (arow) {
      {  // query quarter = bf16(h2 row) · bf16(Wq columns), v_mfma_f32_16x16x32_bf16 with the row in
         // A-row 0 (lanes l & 15 == 0), wave w over k-steps [8w, 8w+8), 2 column tiles; the 8 row
         // fragments in flight at once (one round trip)
        tp_f4 qa[2] = {};
        const auto rs = tp_rsrc(a.H2X);
        const bool r0 = (lane & 15) == 0;
        const int vo = (int)(((long)par * 64 * H + tp_afl(rb, 8 * (lane >> 4), H)) * 2);
        tp_bf8 hf[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) hf[i] = tp_ldx4<true>(rs, vo, (8 * w + i) * 1024);
        tp_wait(hf);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (!r0) hf[i] = tp_bf8{};
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            qa[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[i], wqf[((8 * w + i) * 2 + nt) * 64 + lane], qa[nt], 0, 0, 0);
        if (lane < 16) {
          qps[w * 32 + lane] = qa[0][0];
          qps[w * 32 + 16 + lane] = qa[1][0];
        }
      }
      __syncthreads();
      TP_STAMP(10);
      if (tid < 32) {
        float q = qps[tid];
#pragma unroll
        for (int i = 1; i < TP_NW; ++i) q += qps[i * 32 + tid];
        qv[tid] = q + qbias;
      }
      __syncthreads();
      TP_STAMP(11);
      // energy partials of this quarter: e_j = Σ_a v_a tanh(u_ja), a over the quarter's 32 dims,
      //   u_ja = keys_ja + q_a + b_a + Σ_c f_jc W_loc[c][a],  f_jc = bc_c + Σ_tap cum[j + tap - 15] Kc[tap][c]
      // with the conv folded through W_loc: Σ_c f_jc W_loc[c][a] = Σ_tap cum[j + tap - 15] KW[a][tap] +
      // (bc·W_loc)_a (the bias term is in qv).  U^T[a][j] = Σ_tap KW[a][tap] C[tap][j] on fp32 MFMA
      // (exact fp32 products), C[tap][j] = cum[j + tap - 15] read straight from the zero-padded LDS
      // copy.  The location features themselves (FALL, the backward's operand) are written after the loop.
      {
        const float* thb = a.TH + ((long)t * B + rb) * Tin * A;  // this row's [Tin][A] block of step t
        const tp_f4 q0 = *reinterpret_cast<const tp_f4*>(qv + 4 * g4), q1 = *reinterpret_cast<const tp_f4*>(qv + 16 + 4 * g4);
#pragma unroll
        for (int r = 0; r < NTW; ++r) {
          const int nt = w + 4 * r;
          if (16 * nt >= Tin) break;  // wave-uniform
          const int j = 16 * nt + jl;
          float cb[8];
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) cb[ks] = cw[j + 4 * ks + g4];
          tp_f4 acc[2] = {};
#pragma unroll
          for (int ks = 0; ks < 8; ++ks)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
              acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kwa[8 * mt + ks], cb[ks], acc[mt], 0, 0, 0);
          float e = 0.f;
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const tp_f4 qq = mt ? q1 : q0;
            tp_f4 th4;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              th4[i] = tp_tanh(acc[mt][i] + tp_aget(key[8 * r + 4 * mt + i]) + qq[i]);
              e += vav[4 * mt + i] * th4[i];
            }
            if (j < Tin)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(tp_u4, th4), tp_rsrc(thb),
                                                     (j * A + 32 * sib + 16 * mt + 4 * g4) * 4, 0, 0);
          }
          e += __shfl_xor(e, 16, 64);
          e += __shfl_xor(e, 32, 64);
          if (g4 == 0 && j < Tin) {
            ep[j] = e;
            __builtin_amdgcn_raw_buffer_store_b64(tp_u2{__float_as_uint(e), tag},
                                                  tp_rsrc(a.EX + (((long)par * 64 + rb) * 4 + sib) * TM), j * 8, 0, 16);
          }
        }
      }
    }
    TP_STAMP(12);
    // off-chain terms while the other quarters' energy partials travel
    if (more) {
      if (ocm == 0) {
        hz2_part(t);
      } else {
        hz1_part(t, TP_KSW / 2, TP_KSW);
        if (ocm == 3) hz2_part(t, 0, TP_KSW / 2);
      }
    }
    __syncthreads();  // the own partials in ep[]
    TP_STAMP(13);
    if (arow) {
      // take the other quarters' partials of energy j = tid (granules), sum in quarter order
      if (w < (Tin + 63) / 64) {
        const bool act = tid < Tin;
        const auto rs = tp_rsrc(a.EX + ((long)par * 64 + rb) * 4 * TM);
        float e4[4];
        const float own = act ? ep[tid] : 0.f;
        const bool ok = tp_spin(a, TP_PH_E, [&] {
          bool good = true;
          if (act) {
            unsigned bad = 0u;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              if (s == sib) {
                e4[s] = own;
              } else {
                const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (s * TM + tid) * 8, 0, 16);
                e4[s] = __uint_as_float(x[0]);
                bad |= x[1] ^ tag;
              }
            }
            good = bad == 0u;
          }
          return good;
        });
        if (!ok) sfail[0] = 1;
        if (act) al[tid] = ((e4[0] + e4[1]) + e4[2]) + e4[3];
      }
      __syncthreads();
      TP_STAMP(14);
      if (sfail[0]) return;
      // masked softmax over j < len (attention.py:218, TF _maybe_mask_score), cumulative alignments
      const float ev = tid < len ? al[tid] : -INFINITY;
      const float mx = tp_block_max(ev, scr);
      const float x = tid < len ? __expf(ev - mx) : 0.f;
      const float ssum = tp_block_sum(x, scr);
      if (tid < Tin) {
        const float alv = x * __builtin_amdgcn_rcpf(ssum);
        al[tid] = alv;
        const float cn = cw[15 + tid] + alv;
        cw[15 + tid] = cn;
        if (sib == 0) {
          tp_bst(a.ALIGN + (long)rb * Tin * T, tid * T * 4, t * 4, alv);
          tp_bst(a.ALN + ((long)t * B + rb) * Tin, tid * 4, 0, alv);
          tp_bst(a.CUM + ((long)(t + 1) * B + rb) * Tin, tid * 4, 0, cn);
        }
      }
      __syncthreads();
      TP_STAMP(15);
      // context quarter: channels [256 sib, 256 sib + 256) = Σ_j align_j · values_j (bf16 values;
      // align is 0 past T_in, so the position loop needs no bound)
      float s0 = 0.f, s1 = 0.f;
      const tp_f4* al4 = reinterpret_cast<const tp_f4*>(al + (TM / 2) * vg);
#pragma unroll
      for (int i4 = 0; i4 < TM / 8; ++i4) {
        const tp_f4 wv = al4[i4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned v = __float_as_uint(tp_aget(vals[4 * i4 + e]));
          s0 += wv[e] * tp_lo(v);
          s1 += wv[e] * tp_hi(v);
        }
      }
      cr[vg * 256 + 2 * vcp] = s0;
      cr[vg * 256 + 2 * vcp + 1] = s1;
      __syncthreads();
      const float ctx = cr[tid] + cr[256 + tid];
      cr[tid] = ctx;  // each thread rewrites only its own channel
      __syncthreads();
      TP_STAMP(16);
      if (tid < 32) {
        const float* cs = cr + 8 * tid;
        const tp_u4 v = {tp_pack(cs[0], cs[1]), tp_pack(cs[2], cs[3]), tp_pack(cs[4], cs[5]), tp_pack(cs[6], cs[7])};
        tp_st16(a.CX, (int)(((long)par * 64 * D + tp_afl(rb, 256 * sib + 8 * tid, D)) * 2), v);
      }
      tp_publish(a, TP_PH_CTX, tag);
      TP_STAMP(17);
      {
        const long i = (long)t * B + rb;
        tp_bst(a.PIN + i * (H + D), (H + 256 * sib + tid) * 4, 0, ctx);
        tp_bst(a.X1 + (i + B) * LX1, (P + 256 * sib + tid) * 4, 0, ctx);
      }
    }
    // off-chain terms while the contexts travel
    if (more) {
      if (ocm != 0) hz2_part(t, ocm == 3 ? TP_KSW / 2 : 0, TP_KSW);
      if (ocm != 2) prenet_part(t + 1);
    }
    TP_STAMP(18);
  }
#undef TP_STAMP
  if (g == 0 && tid == 0) a.ctl[1] = T;
}

__global__ void k_tp_prenet_rows(const float* __restrict__ X1, long ld, int B, int T, __bf16* __restrict__ preh) {
  const long n = (long)T * 64 * TP_P;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int t = (int)(i / (64 * TP_P)), rem = (int)(i % (64 * TP_P)), r = rem / TP_P, k = rem % TP_P;
    preh[(long)t * 64 * TP_P + tp_afl(r, k, TP_P)] = r < B ? (__bf16)X1[((long)t * B + r) * ld + k] : (__bf16)0.f;
  }
}

__global__ __launch_bounds__(256) void k_tp_kwt(const float* __restrict__ Kc, const float* __restrict__ bc,
                                                const float* __restrict__ Wl, float* __restrict__ KWT) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (a, tap)
  if (i >= TP_A * 32) return;
  const int a = i >> 5, tp = i & 31;
  float acc = 0.f;
  for (int c = 0; c < TP_F; ++c) acc += (tp < TP_KW ? Kc[tp * TP_F + c] : tp == 31 ? bc[c] : 0.f) * Wl[c * TP_A + a];
  KWT[i] = acc;
}

void tp_prepare(const float* Kc, const float* bc, const float* Wl, float* KWT, hipStream_t s) {
  hipLaunchKernelGGL(k_tp_kwt, dim3(TP_A * 32 / 256), dim3(256), 0, s, Kc, bc, Wl, KWT);
  TT2_HIP(hipGetLastError());
}

// one thread per (step, row, position, filter): the 32 filters of a position are 32 adjacent lanes
// (coalesced stores), the cum window is shared through L1
__global__ __launch_bounds__(256) void k_tp_fall(const float* __restrict__ CUM, const float* __restrict__ Kc,
                                                 const float* __restrict__ bc, long npos, int Tin,
                                                 float* __restrict__ FALL) {
  __shared__ float kcs[TP_KW * TP_F + TP_F];
  for (int i = threadIdx.x; i < TP_KW * TP_F; i += blockDim.x) kcs[i] = Kc[i];
  if (threadIdx.x < TP_F) kcs[TP_KW * TP_F + threadIdx.x] = bc[threadIdx.x];
  __syncthreads();
  constexpr int pad = (TP_KW - 1) / 2;
  const long n = npos * TP_F;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i & (TP_F - 1));
    const long pos = i >> 5;                   // (t, b) row-block * Tin + j
    const int j = (int)(pos % Tin);
    const float* cum = CUM + (pos - j);        // CUM[t][b][0..Tin)
    float acc = kcs[TP_KW * TP_F + c];
    for (int tp = 0; tp < TP_KW; ++tp) {
      const int jj = j + tp - pad;
      acc += ((jj >= 0 && jj < Tin) ? cum[jj] : 0.f) * kcs[tp * TP_F + c];
    }
    FALL[i] = acc;
  }
}

void tp_location_features(const float* CUM, const float* Kc, const float* bc, int B, int T, int Tin, float* FALL,
                          hipStream_t s) {
  static_assert(TP_F == 32, "k_tp_fall: one lane per filter");
  hipLaunchKernelGGL(k_tp_fall, dim3(4096), dim3(256), 0, s, CUM, Kc, bc, (long)T * B * Tin, Tin, FALL);
  TT2_HIP(hipGetLastError());
}

void tp_prenet_rows(const float* X1, long ld, int B, int T, __bf16* preh, hipStream_t s) {
  hipLaunchKernelGGL(k_tp_prenet_rows, dim3(2048), dim3(256), 0, s, X1, ld, B, T, preh);
  TT2_HIP(hipGetLastError());
}

bool tp_device_ok(int dev) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
  if (prop.multiProcessorCount < TP_NB) return false;
  const void* k = reinterpret_cast<const void*>(k_tr_persist);
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tp_lds_bytes()) != hipSuccess)
    return false;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tr_persist, TP_NT, tp_lds_bytes()) != hipSuccess) return false;
  return nb >= 1;
}

// Cooperative launch: the runtime guarantees all TP_NB work-groups are resident at once (or fails
// the launch); the spin-waits depend on it.
void tp_launch(const TpArgs& a, hipStream_t s) {
  TpArgs arg = a;
  void* params[] = {&arg};
  TT2_HIP(launch_persistent(reinterpret_cast<const void*>(k_tr_persist), dim3(TP_NB), dim3(TP_NT), params,
                            (unsigned)tp_lds_bytes(), s));
}

}  // namespace tt2
