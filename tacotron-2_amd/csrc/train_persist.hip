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
#include "train_persist.h"

#ifndef TP_V_ASMLD
#define TP_V_ASMLD 1
#endif
#ifndef TP_V_BST
#define TP_V_BST 1
#endif
#ifndef TP_V_ZMBUF
#define TP_V_ZMBUF 1
#endif
#ifndef TP_V_AGPR
#define TP_V_AGPR 1
#endif

namespace tt2 {

typedef __bf16 tp_bf8 __attribute__((ext_vector_type(8)));
typedef unsigned tp_u2 __attribute__((ext_vector_type(2)));
typedef unsigned tp_u4 __attribute__((ext_vector_type(4)));
typedef float tp_f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned tp_gu32;
typedef __attribute__((address_space(1))) int tp_gi32;
typedef __attribute__((address_space(1))) unsigned long long tp_gu64;
#define TP_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
constexpr long long TP_TIMEOUT = 200000000LL;  // 2 s of s_memrealtime (100 MHz)
enum { TP_PH_H1 = 0, TP_PH_H2 = 1, TP_PH_CTX = 2, TP_PH_E = 3 };
constexpr int TP_NW = TP_NT / 64;          // waves
constexpr int TP_KSW = 32 / TP_NW;         // k-steps per wave of a 1024-deep segment
constexpr int TP_PKW = TP_P / 32 / TP_NW;  // prenet k-steps per wave
constexpr int TP_RG = TP_NT / 32;          // attention row groups (32 dims each)
constexpr int TP_VG = TP_NT / 128;         // context row groups (128 channel pairs each)
static_assert(TP_KSW % 4 == 0 && TP_PKW >= 1 && TP_H == 1024 && TP_D == 1024, "train_persist geometry");

// LDS layout (floats)
constexpr int TP_KW = 31;                       // attention_kernel (fork default; tr_persist_fits)
constexpr int TP_JB = TP_TMAX / 8;              // encoder positions per row group (8 groups of 32 lanes)
constexpr int TPL_RED = 0;                      // [TP_NW waves][64][16] partial gate tiles
constexpr int TPL_OC1 = TPL_RED + TP_NW * 1024; // [64][16] off-chain LSTM-1 terms of the next step
constexpr int TPL_OC2 = TPL_OC1 + 1024;         // [64][16] off-chain LSTM-2 terms
constexpr int TPL_WQ = TPL_OC2 + 1024;          // query columns of this quarter as bf16 B fragments
constexpr int TPL_F = TPL_WQ + TP_H * 32 / 2;   // [TMAX][32] location features
constexpr int TPL_CW = TPL_F + TP_TMAX * 32;    // [15 + TMAX + 17 + 16] cumulative alignments, zero padded
constexpr int TPL_KC = TPL_CW + TP_TMAX + 48;   // [32 taps][32] location conv kernel (zero padded)
constexpr int TPL_WL = TPL_KC + 32 * 32;        // [F][32] location_features_layer columns of this quarter
constexpr int TPL_QP = TPL_WL + TP_F * 32;      // [TP_NW][32] query partials
constexpr int TPL_QV = TPL_QP + TP_NW * 32;     // [32] q + b_a
constexpr int TPL_EP = TPL_QV + 32;             // [TMAX] this quarter's energy partials
constexpr int TPL_AL = TPL_EP + TP_TMAX;        // [TMAX] energies -> alignments (zero past T_in)
constexpr int TPL_CR = TPL_AL + TP_TMAX;        // [TP_VG][256] context partials
constexpr int TPL_SC = TPL_CR + TP_VG * 256;    // [16] reduction scratch, then ints
constexpr int TPL_END = TPL_SC + 32;
static_assert(TP_TMAX % 32 == 0 && TP_VG == 2, "train_persist attention geometry");

size_t tp_lds_bytes() { return sizeof(float) * (size_t)TPL_END; }

__device__ __forceinline__ float tp_sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float tp_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float tp_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ unsigned tp_pack(float lo, float hi) {
  return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)lo) |
         ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)hi) << 16);
}
// explicit AGPR residency for the per-row constants the attention reads once per step (keys, the
// values quarter): the VGPRs stay free for the LSTM products' fragments in flight
__device__ __forceinline__ float tp_aput(float v) {
#if !TP_V_AGPR
  return v;
#endif
  float r;
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(r) : "v"(v));
  return r;
}
__device__ __forceinline__ float tp_aget(float r) {
#if !TP_V_AGPR
  return r;
#endif
  float v;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(r));
  return v;
}

// sc1 (L1-bypassing) loads and write-through stores of exchanged data; offsets in bytes
__device__ __forceinline__ auto tp_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// plain buffer store / load of one dword: per-lane byte offset + uniform byte offset (no per-lane
// 64-bit addresses in the step loop, where the compiler would keep one per store site alive)
__device__ __forceinline__ void tp_bst(const void* base, int vbyte, int sbyte, float v) {
#if !TP_V_BST
  *reinterpret_cast<float*>(reinterpret_cast<char*>(const_cast<void*>(base)) + vbyte + sbyte) = v;
  return;
#endif
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), tp_rsrc(base), vbyte, sbyte, 0);
}
__device__ __forceinline__ void tp_st8(void* base, int byte_off, tp_u2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, tp_rsrc(base), byte_off, 0, 16);
}
__device__ __forceinline__ void tp_st16(void* base, int byte_off, tp_u4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, tp_rsrc(base), byte_off, 0, 16);
}

// Wave-uniform bounded spin until cond() holds on every lane; false on timeout or a peer's failure
// (ctl[0] != 0), the failing phase recorded there.
template <class F>
__device__ __forceinline__ bool tp_spin(const TpArgs& a, int ph, F cond) {
  long long t0 = 0;
  for (unsigned spin = 0;; ++spin) {
    if (__all(cond())) return true;
    if ((spin & 63) == 0) {
      const long long now = __builtin_amdgcn_s_memrealtime();
      if (spin == 0) {
        t0 = now;
      } else if (__hip_atomic_load((tp_gi32*)a.ctl, TP_RLX) != 0 || now - t0 > TP_TIMEOUT) {
        if ((threadIdx.x & 63) == 0) __hip_atomic_store((tp_gi32*)a.ctl, 1 + ph, TP_RLX);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ unsigned tp_flag(const unsigned* f) {
  return __hip_atomic_load((tp_gu32*)const_cast<unsigned*>(f), TP_RLX);
}
// wave poll: flags of producers [base, base + n) of phase ph reached tag (this XCD group's replica)
__device__ __forceinline__ bool tp_poll(const TpArgs& a, int ph, int base, int n, unsigned tag) {
  const unsigned* f = a.flags + ((long)ph * TP_NREP + (blockIdx.x & (TP_NREP - 1))) * TP_NB + base;
  const int lane = threadIdx.x & 63;
  return tp_spin(a, ph, [&] { return lane >= n || tp_flag(f + lane) >= tag; });
}
// every wave drains its stores, one barrier, then this work-group's flag in every replica
__device__ __forceinline__ void tp_publish(const TpArgs& a, int ph, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < TP_NREP)
    __hip_atomic_store((tp_gu32*)(a.flags + ((long)ph * TP_NREP + threadIdx.x) * TP_NB + blockIdx.x), tag, TP_RLX);
}

// wave partial tiles (4 row tiles x 16 columns) -> red[w][64][16]
__device__ __forceinline__ void tp_put_tiles(float* red, const tp_f4 (&acc)[4], int w, int lane) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w * 1024 + (16 * mt + 4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[mt][r];
}

// 16-byte buffer load issued by inline asm: the compiler schedules at most two of its own loads
// ahead of their MFMAs here (measured: one round trip per fragment), so a batch of fragments is
// issued back to back and waited for once (tp_wait), one L2 round trip per batch
template <bool SC1>
__device__ __forceinline__ tp_bf8 tp_ldx4(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
  tp_bf8 r;
#if !TP_V_ASMLD
  return __builtin_bit_cast(tp_bf8, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, SC1 ? 16 : 0));
#endif
  if constexpr (SC1)
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen sc1" : "=v"(r) : "v"(vo), "s"(rs), "s"(so) : "memory");
  else
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(r) : "v"(vo), "s"(rs), "s"(so) : "memory");
  return r;
}
// wait for every load of the batch; the fragments pass through as operands so no use is scheduled
// above the wait
template <int N>
__device__ __forceinline__ void tp_wait(tp_bf8 (&f)[N]) {
#if TP_V_ASMLD
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
#endif
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
  float* const oc1 = sm + TPL_OC1;
  float* const oc2 = sm + TPL_OC2;
  tp_bf8* const wqf = reinterpret_cast<tp_bf8*>(sm + TPL_WQ);
  float* const fs = sm + TPL_F;
  float* const cw = sm + TPL_CW;
  float* const kcs = sm + TPL_KC;
  float* const wls = sm + TPL_WL;
  float* const qps = sm + TPL_QP;
  float* const qv = sm + TPL_QV;
  float* const ep = sm + TPL_EP;
  float* const al = sm + TPL_AL;
  float* const cr = sm + TPL_CR;
  float* const scr = sm + TPL_SC;
  int* const sfail = reinterpret_cast<int*>(sm + TPL_SC + 16);
  constexpr int H = TP_H, P = TP_P, D = TP_D, A = TP_A, LX1 = TP_LX1, TM = TP_TMAX, JB = TP_JB;
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
  const int wcol = (fn >> 2) * H + 4 * g + (fn & 3);
  const int wvo1 = (wcol * LX1 + fk) * 2, wvo2 = (wcol * 2 * H + fk) * 2;  // bytes (K1T / K2T < 2 GB)
  const int wk0 = 32 * TP_KSW * w;
#pragma unroll
  for (int i = 0; i < TP_KSW; ++i) {
    w1c[i] = *reinterpret_cast<const tp_bf8*>(a.K1T + (long)wcol * LX1 + P + wk0 + 32 * i + fk);
    w2i[i] = *reinterpret_cast<const tp_bf8*>(a.K2T + (long)wcol * 2 * H + wk0 + 32 * i + fk);
  }
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

  // ---- attention row constants.  Thread (aa = tid & 31, grp = tid >> 5): attention dim / filter aa
  // of this quarter, encoder positions [JB grp, JB grp + JB) (location features, energies); context:
  // channel pair vcp, positions [TM/2 vg, TM/2 vg + TM/2)
  const int aa = tid & 31, grp = tid >> 5, adim = 32 * sib + aa;
  const int vcp = tid & 127, vg = tid >> 7;
  float key[JB];          // AGPRs: keys[rb][JB grp + i][adim]
  float vals[TM / 2];     // AGPRs: bf16 pairs of values16[rb][TM/2 vg + i][256 sib + 2 vcp]
#pragma unroll
  for (int i = 0; i < JB; ++i) {
    const int j = JB * grp + i;
    key[i] = tp_aput((arow && j < Tin) ? a.keys[((long)rb * Tin + j) * A + adim] : 0.f);
  }
#pragma unroll
  for (int i = 0; i < TM / 2; ++i) {
    const int j = (TM / 2) * vg + i;
    const unsigned v = (arow && j < Tin)
                           ? *reinterpret_cast<const unsigned*>(a.values16 + ((long)rb * Tin + j) * D + 256 * sib + 2 * vcp)
                           : 0u;
    vals[i] = tp_aput(__uint_as_float(v));
  }
  float vav = 0.f, bav = 0.f, bcv = 0.f;
  int len = 0;
  if (arow) {
    vav = a.va[adim];
    bav = a.ba[adim];
    bcv = a.bc[aa];
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
    for (int e = tid; e < 32 * 32; e += TP_NT) kcs[e] = (e >> 5) < TP_KW ? a.Kc[(e >> 5) * TP_F + (e & 31)] : 0.f;
    for (int e = tid; e < TP_F * 32; e += TP_NT) wls[e] = a.Wl[(e >> 5) * A + 32 * sib + (e & 31)];
  }
  for (int e = tid; e < TM + 48; e += TP_NT) cw[e] = 0.f;
  for (int e = tid; e < TM; e += TP_NT) al[e] = 0.f;
  if (tid == 0) sfail[0] = 0;

  // ---- off-chain products: wave partials -> red, summed into dst[64][16]
  auto reduce_into = [&](float* dst, const tp_f4 (&acc)[4]) {
    tp_put_tiles(red, acc, w, lane);
    __syncthreads();
    for (int e = tid; e < 1024; e += TP_NT) {
      float s = red[e];
#pragma unroll
      for (int ww = 1; ww < TP_NW; ++ww) s += red[ww * 1024 + e];
      dst[e] = s;
    }
    __syncthreads();
  };
  // LSTM-1 terms of step tn: prenet_tn·W1p (+ hz1_{tn-1}·W1h, parity (tn-1) & 1)
  auto offchain1 = [&](int tn) {
    tp_f4 acc[4] = {};
    tp_mfma_stream<TP_PKW, false>(acc, a.preh + (long)tn * 64 * P, P, TP_PKW * w, a.K1T, wvo1, 32 * TP_PKW * w, lane);
    if (tn > 0) {
#pragma unroll
      for (int c = 0; c < TP_KSW; c += 4)
        tp_mfma_stream<4, true>(acc, a.Z1X + (long)((tn - 1) & 1) * 64 * H, H, TP_KSW * w + c, a.K1T, wvo1,
                                P + D + wk0 + 32 * c, lane);
    }
    reduce_into(oc1, acc);
  };
  // LSTM-2 terms of step tn: hz2_{tn-1}·W2h
  auto offchain2 = [&](int tn) {
    tp_f4 acc[4] = {};
#pragma unroll
    for (int c = 0; c < TP_KSW; c += 4)
      tp_mfma_stream<4, true>(acc, a.Z2X + (long)((tn - 1) & 1) * 64 * H, H, TP_KSW * w + c, a.K2T, wvo2, H + wk0 + 32 * c,
                              lane);
    reduce_into(oc2, acc);
  };
  offchain1(0);  // hz1_{-1} = 0
  for (int e = tid; e < 1024; e += TP_NT) oc2[e] = 0.f;
  __syncthreads();

  // one LSTM layer's epilogue for thread (er, eu): gates = bias + off-chain + Σ wave partials
  // (k_tr_fused<TF_FWD>'s cell + zoneout, Architecture_wrappers.py:214-224 / modules.py:236-244)
  struct Cell {
    float si, tj, sf, so, cn, hn, cz, hz;
  };
  auto cell = [&](const float* oc, const float (&bias)[4], float cp, float hp, float kc, float kh) {
    float pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ci = er * 16 + 4 * q + eu;
      float s = red[ci];
#pragma unroll
      for (int ww = 1; ww < TP_NW; ++ww) s += red[ww * 1024 + ci];
      pre[q] = bias[q] + (oc[ci] + s);
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
#if !TP_V_ZMBUF
      const uint8_t* zp = a.zm + (long)t * 4 * B * H + evo;
      kc1 = (float)zp[0];
      kh1 = (float)zp[zs];
      kc2 = (float)zp[2 * zs];
      kh2 = (float)zp[3 * zs];
      (void)rz;
#else
      kc1 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, 0, 0);
      kh1 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, zs, 0);
      kc2 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, 2 * zs, 0);
      kh2 = (float)__builtin_amdgcn_raw_buffer_load_b8(rz, evo, 3 * zs, 0);
#endif
    }
    // ================= L1: ctx_{t-1}·W1c (wave w: context k of quarter (TP_KSW w) / 8)
    {
      tp_f4 acc[4] = {};
      if (t > 0) {
        if (!tp_poll(a, TP_PH_CTX, 64 * ((TP_KSW * w) >> 3), B, tag - 1u)) sfail[0] = 1;
        TP_STAMP(1);
        tp_mfma_seg(acc, a.CX + (long)((t - 1) & 1) * 64 * D, D, TP_KSW * w, w1c, lane);
      }
      tp_put_tiles(red, acc, w, lane);
      TP_STAMP(2);
      __syncthreads();
      TP_STAMP(3);
      if (sfail[0]) return;
      Cell o{};
      if (eth) o = cell(oc1, bias1, c1, hz1, kc1, kh1);
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
        c1 = o.cz;
        hz1 = o.hz;
      }
    }
    // ================= L2: h1_t·W2i (wave w: k-steps [TP_KSW w, TP_KSW (w+1)) = producers [8 TP_KSW w, ..))
    {
      tp_f4 acc[4] = {};
      if (!tp_poll(a, TP_PH_H1, 8 * TP_KSW * w, 8 * TP_KSW, tag)) sfail[0] = 1;
      TP_STAMP(5);
      tp_mfma_seg(acc, a.H1X + (long)par * 64 * H, H, TP_KSW * w, w2i, lane);
      tp_put_tiles(red, acc, w, lane);
      TP_STAMP(6);
      __syncthreads();
      if (sfail[0]) return;
      Cell o{};
      if (eth) o = cell(oc2, bias2, c2, hz2, kc2, kh2);
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
        c2 = o.cz;
        hz2 = o.hz;
      }
    }
    // ================= H2 of every producer (wave w polls its 8 TP_KSW producers), then the attention row
    if (!tp_poll(a, TP_PH_H2, 8 * TP_KSW * w, 8 * TP_KSW, tag)) sfail[0] = 1;
    __syncthreads();
    TP_STAMP(8);
    if (sfail[0]) return;
    const bool more = t + 1 < T;
    if (arow) {
      {  // query quarter = bf16(h2 row) · bf16(Wq columns), v_mfma_f32_16x16x32_bf16 with the row in
         // A-row 0 (lanes l & 15 == 0), wave w over k-steps [8w, 8w+8), 2 column tiles
        tp_f4 qa[2] = {};
        const auto rs = tp_rsrc(a.H2X);
        const bool r0 = (lane & 15) == 0;
        const int vo = r0 ? (int)(((long)par * 64 * H + tp_afl(rb, 8 * (lane >> 4), H)) * 2) : 0;
        tp_bf8 hf[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          hf[i] = __builtin_bit_cast(tp_bf8, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (8 * w + i) * 1024, 16));
          if (!r0) hf[i] = tp_bf8{};
        }
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
      {  // location features of positions [JB grp, JB grp + JB), filter aa: the tap window in registers
        float kc[TP_KW], win[JB + TP_KW - 1];
#pragma unroll
        for (int tp = 0; tp < TP_KW; ++tp) kc[tp] = kcs[tp * 32 + aa];
#pragma unroll
        for (int i = 0; i < JB + TP_KW - 1; ++i) win[i] = cw[JB * grp + i];  // cw[15 + j] = cum[j], pad 15
#pragma unroll
        for (int jj = 0; jj < JB; ++jj) {
          float f = bcv;
#pragma unroll
          for (int tp = 0; tp < TP_KW; ++tp) f += win[jj + tp] * kc[tp];
          const int j = JB * grp + jj;
          fs[j * 32 + aa] = f;
          if (sib == 0 && j < Tin) tp_bst(a.FALL + ((long)t * B + rb) * Tin * TP_F, (JB * grp * TP_F + aa) * 4, jj * TP_F * 4, f);
        }
      }
      __syncthreads();
      TP_STAMP(10);
      if (tid < 32) {
        float q = qps[tid];
#pragma unroll
        for (int i = 1; i < TP_NW; ++i) q += qps[i * 32 + tid];
        qv[tid] = q + bav;
      }
      __syncthreads();
      TP_STAMP(11);
      {  // energy partials of this quarter: e_j = Σ_{a in quarter} v_a·tanh(keys + q + b_a + f·W_loc)
        const float qb = qv[aa];
        float wl[TP_F];
#pragma unroll
        for (int c = 0; c < TP_F; ++c) wl[c] = wls[c * 32 + aa];
        const float* thb = a.TH + ((long)t * B + rb) * Tin * A;  // this row's [Tin][A] block of step t
        const auto rge = tp_rsrc(a.EX + (((long)par * 64 + rb) * 4 + sib) * TM);
#pragma unroll
        for (int i = 0; i < JB; ++i) {
          const int j = JB * grp + i;
          if (j < Tin) {
            float u = tp_aget(key[i]) + qb;
            const tp_f4* fr = reinterpret_cast<const tp_f4*>(fs + j * 32);
#pragma unroll
            for (int c4 = 0; c4 < 8; ++c4) {
              const tp_f4 fv = fr[c4];
#pragma unroll
              for (int e = 0; e < 4; ++e) u += fv[e] * wl[4 * c4 + e];
            }
            const float th = tanhf(u);
            tp_bst(thb, (JB * grp * A + adim) * 4, i * A * 4, th);
            float e = vav * th;
#pragma unroll
            for (int o = 16; o >= 1; o >>= 1) e += __shfl_xor(e, o, 64);
            if (aa == 0) {
              ep[j] = e;
              __builtin_amdgcn_raw_buffer_store_b64(tp_u2{__float_as_uint(e), tag}, rge, JB * grp * 8, i * 8, 16);
            }
          }
        }
      }
    }
    TP_STAMP(12);
    // off-chain LSTM-1 terms of t+1 while the other quarters' energy partials travel
    if (more) offchain1(t + 1);
    else __syncthreads();  // the own partials in ep[] (offchain1's barriers order them otherwise)
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
      const float x = tid < len ? expf(ev - mx) : 0.f;
      const float ssum = tp_block_sum(x, scr);
      if (tid < Tin) {
        const float alv = x / ssum;
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
    // off-chain LSTM-2 terms of t+1 (needed only after the next context)
    if (more) offchain2(t + 1);
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
