// Wide-channel WaveNet generator for MI355X (gfx950): WaveNet.incremental (wavenet.py:821-886) with
// R = 128 (fork default, hparams.py:222-239) or R = 256 (paper default, paper_hparams.py:199-204).
//
// At R=64 one CU holds three layers in registers (k_generate_pipe, wavenet.hip).  A layer at R=128
// is 0.5 MB of fp32 weights (dilated conv 3R x 2R + skip/out R x 2R), at R=256 2 MB -- more than
// one CU's 512 KB register file.  So each layer is split over NC = 2 / 8 work-groups by GATE
// COLUMNS: work-group c owns the gate pairs (a_i, b_i) of z channels [c·R/NC, (c+1)·R/NC), i.e. a
// contiguous block of the gate-permuted columns, computes its slice of z = tanh(a)·σ(b) and the
// partial skip/out 1x1 products of that z slice, and publishes them as data-tagged granules
// {tag = t+1, fp32} (the data is the flag; MI355X_MICROARCH.md Guideline 16 R2).  The next layer's
// work-groups sum the NC partials (work-group 0 folds in the biases, the residual and the running
// skip sum, and the legacy sqrt(1/2) scalings, which are linear) -- one hand-off per layer.  A
// head work-group runs ReLU -> 1x1 -> ReLU -> 1x1 and the MoL / Gaussian sampler and hands the
// sample back to layer 0.  Per lane: 32x4 tap weights + 16x4 x(t) weights + 16x4 skip/out weights
// = 256 registers (VGPR + AGPR at one wave per SIMD).
//
// The fast-WaveNet queues (2d+1 rows of R, up to d = 512 at 10 layers per stack) exceed the LDS,
// so every work-group keeps a private copy of its layer's queue in global memory (L2-resident):
// written with plain stores, read back with L1-bypassing sc1 loads after the storing wave drained
// -- the same CU only, so no cross-CU visibility is involved.  The taps x(t-2d), x(t-d) are read
// and multiplied before the sample's input arrives (off the serial chain).
#include "wavenet_wide.h"

#include <algorithm>
#include <cstdlib>

namespace tt2 {

typedef __attribute__((address_space(1))) unsigned long long ww_gu64;
typedef __attribute__((address_space(1))) int ww_gi32;

__device__ __forceinline__ void ww_put(unsigned long long* g, unsigned tag, float v) {
  __hip_atomic_store((ww_gu64*)g, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ww_get(const unsigned long long* g) {
  return __hip_atomic_load((ww_gu64*)const_cast<unsigned long long*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ f32x4 ww_ld4(const float* base, long i4) {  // sc1: bypass L1, L2-served
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i4 * 16), 0, 16));
}

// Bounded wave-uniform spin until ok() holds on every lane; false on timeout (4 s) or a peer's
// failure (status word), which is then recorded.
template <class F>
__device__ __forceinline__ bool ww_spin(int* status, int lane, F ok) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned it = 0;; ++it) {
    if (__all(ok())) return true;
    if ((it & 255) == 255) {
      if (__hip_atomic_load((ww_gi32*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
        if (lane == 0) __hip_atomic_store((ww_gi32*)status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
}

// Sum over N adjacent lanes (N <= 16, a power of two); every lane of the group ends with the sum.
template <int N>
__device__ __forceinline__ void ww_reduce(f32x4& a) {
#define TT2_STEP(C)                                                                                  \
  {                                                                                                  \
    const float t0 = dpp_f<C>(a[0]), t1 = dpp_f<C>(a[1]), t2 = dpp_f<C>(a[2]), t3 = dpp_f<C>(a[3]); \
    a[0] += t0; a[1] += t1; a[2] += t2; a[3] += t3;                                                  \
  }
  if (N >= 2) TT2_STEP(DPP_XOR1)
  if (N >= 4) TT2_STEP(DPP_XOR2)
  if (N >= 8) TT2_STEP(DPP_HALF_MIRROR)
  if (N >= 16) TT2_STEP(DPP_MIRROR)
#undef TT2_STEP
}

// gate nonlinearities on v_exp_f32 + v_rcp_f32 (common.h tanh_rcp / sigm_fast: abs error < 3e-7,
// no IEEE division on the per-layer chain)
__device__ __forceinline__ float ww_tanh(float x) { return tanh_rcp(x); }
__device__ __forceinline__ float ww_sigm(float x) { return sigm_fast(x); }

// two v_pk_fma_f32 (x broadcast through op_sel_hi) instead of four v_fma_f32: the per-layer
// gate and [out | skip] products sit on the sample chain, so halving their issue count counts
typedef float f32x2 __attribute__((ext_vector_type(2)));
#ifndef WW_PK
#define WW_PK 1
#endif
__device__ __forceinline__ void ww_fma4(f32x4& acc, float x, const f32x4& w) {
  if (!WW_PK) { acc[0] += x * w[0]; acc[1] += x * w[1]; acc[2] += x * w[2]; acc[3] += x * w[3]; return; }
  const f32x2 xx = {x, x};
  const f32x2 lo = __builtin_elementwise_fma(xx, f32x2{w[0], w[1]}, f32x2{acc[0], acc[1]});
  const f32x2 hi = __builtin_elementwise_fma(xx, f32x2{w[2], w[3]}, f32x2{acc[2], acc[3]});
  acc = f32x4{lo[0], lo[1], hi[0], hi[1]};
}
__device__ __forceinline__ void ww_fma4s(f32x4& acc, float x, const f32x4& w) {
  acc[0] += x * w[0]; acc[1] += x * w[1]; acc[2] += x * w[2]; acc[3] += x * w[3];
}
#ifndef WW1_PK
#define WW1_PK 0
#endif
__device__ __forceinline__ void ww1_fma4(f32x4& acc, float x, const f32x4& w) {
  if (WW1_PK) ww_fma4(acc, x, w); else ww_fma4s(acc, x, w);
}

template <bool GAUSS>
__device__ void ww1_layer(const WideArgs& a, float* sm, const unsigned long long* sample_gran);

template <int R, bool GAUSS, bool ONEHOP = false>
__global__ __launch_bounds__(WW_THREADS, 1) void k_generate_wide(WideArgs a) {
  constexpr int NC = ww_nc(R), S = R, G = 2 * R, ZC = R / NC, GC = 2 * ZC, NQ = GC / 4, NKS = WW_THREADS / NQ;
  // TWO_HOP (R = 256): work-group c gathers the whole z (an all-gather of the layer's NC z slices)
  // and produces COMPLETE outputs for its slice of OC = OUT / NC columns of [skip | out] -- two
  // small hops per layer (256 z granules, then <= 320 output granules per consumer) instead of
  // every consumer summing NC partial rows of OUT (4096 granules, 32 KB per consumer and layer)
  constexpr bool TWO_HOP = NC == 8;
  constexpr int OUT = S + R, OC = TWO_HOP ? OUT / NC : OUT, NQ2 = OC / 4, NKS2 = WW_THREADS / NQ2;
  constexpr int NG = NC * OUT;
  static_assert(2 * R / NKS == WW_TAPK && R / NKS == WW_XK && (TWO_HOP ? R : ZC) / NKS2 == WW_SOK,
                "k-slice geometry");
  static_assert(!TWO_HOP || (R == WW_THREADS && OC == 64 && S % OC == 0), "two-hop geometry: R = 256");
  const float SQH = 0.70710677f;  // float32(np.sqrt(0.5))
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L;
  unsigned long long* const sample_gran = ONEHOP ? a.gran + (long)(L + 1) * W1_GB : a.gran + (long)L * NG;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  int* flag = reinterpret_cast<int*>(sm);
  if (tid == 0) flag[0] = 0;

  if ((int)blockIdx.x == (ONEHOP ? (L + 1) * NC : L * NC)) {
    // ======================= head: ReLU -> 1x1 -> ReLU -> 1x1 -> sampler =======================
    constexpr int NQH = S / 4, NKSH = WW_THREADS / NQH, HK = S / NKSH;
    float* skv = sm + 16;          // [S] relu(skips)
    float* h1 = skv + S;           // [S]
    float* lg = h1 + S;            // [32]
    float* gum = lg + 32;          // [2][16] Gumbel terms (+ [15] logistic / normal draw) by t&1
    const int qh = tid / NKSH, kh = tid % NKSH;
    // f2 in registers: column quad cq = tid / 32, rows k = i * 32 + ks (ks = tid % 32) -- the
    // 32 row slices of one quad sit in one half-wave and reduce on DPP
    constexpr int RK = S / 32;
    static_assert(S % 32 == 0 && WW_THREADS == 256, "head f2 geometry");
    const int cq = tid >> 5, ks = tid & 31;
    f32x4 w2[RK];
#pragma unroll
    for (int i = 0; i < RK; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cc = cq * 4 + e;
        w2[i][e] = cc < a.C ? a.f2_w[(i * 32 + ks) * a.C + cc] : 0.f;
      }
    f32x4 w1[HK];
#pragma unroll
    for (int i = 0; i < HK; ++i) w1[i] = reinterpret_cast<const f32x4*>(a.f1_w + (long)(kh * HK + i) * S)[qh];
    const f32x4 b1 = reinterpret_cast<const f32x4*>(a.f1_b)[qh];
    f32x4 b2;
#pragma unroll
    for (int e = 0; e < 4; ++e) b2[e] = cq * 4 + e < a.C ? a.f2_b[cq * 4 + e] : 0.f;
    const int nr = a.C / 3;
    // one-hop: the tail's skip block, read at [256 + tid] like the two-hop layer's x granules
    const unsigned long long* gin = ONEHOP ? a.gran + (long)L * W1_GB + 2 * R - 256 : a.gran + (long)(L - 1) * NG;
    // layer 0 in the head (ONEHOP, a.l0): thread j owns z channel j; its a / b gate columns sit at
    // gate-permuted pa, pa + 2 of the conditioning; it publishes z_0(s) and x_0(s) with tag s + 1
    const bool fuse0 = ONEHOP && a.l0 != nullptr;
    f32x4 u0a = {0.f, 0.f, 0.f, 0.f}, v0a = u0a, u0b = u0a, v0b = u0a;
    float fwj = 0.f, fbj = 0.f, in1 = 0.f, in2 = 0.f, base_a = 0.f, base_b = 0.f;
    const int pa = 4 * (tid >> 1) + (tid & 1);
    const float* cond0 = a.cond + (long)a.b * a.T * L * (2 * R) + pa;
    if (fuse0) {
      const f32x4* l0 = reinterpret_cast<const f32x4*>(a.l0) + tid * 4;
      u0a = l0[0]; v0a = l0[1]; u0b = l0[2]; v0b = l0[3];
      fwj = a.first_w[tid]; fbj = a.first_b[tid];
      // s = 0: no live taps, x_0(0) = fb
      const float za = u0a[3] + cond0[0] + v0a[2], zb = u0b[3] + cond0[2] + v0b[2];
      ww_put(a.gran + tid, 1u, ww_tanh(za) * ww_sigm(zb));
      ww_put(a.gran + R + tid, 1u, fbj);
    }
    __syncthreads();
    for (int t = 0; t < a.T; ++t) {
      const int cb = t & 1;
      if (fuse0 && t + 1 < a.T) {  // layer 0 at s = t + 1 up to the y_t term, before the skips arrive
        const float* cs = cond0 + (long)(t + 1) * L * (2 * R);
        base_a = u0a[3] + cs[0] + in1 * u0a[1] + v0a[1] + v0a[2];
        base_b = u0b[3] + cs[2] + in1 * u0b[1] + v0b[1] + v0b[2];
        if (t >= 1) {
          base_a += in2 * u0a[0] + v0a[0];
          base_b += in2 * u0b[0] + v0b[0];
        }
      }
      if (wave == 1) {  // this sample's noise (injected, or the device RNG of common.h)
        if (GAUSS) {
          if (lane == 15) gum[cb * 16 + 15] = a.u_log ? a.u_log[(long)t * a.Bg + a.b] : wn_gauss(a.seed, t, a.Bg, a.b);
        } else if (lane < nr) {
          const float um = a.u_mix ? a.u_mix[((long)t * a.Bg + a.b) * nr + lane] : wn_uniform(a.seed, t, a.Bg, a.b, lane);
          gum[cb * 16 + lane] = (float)log(-log((double)um));
        } else if (lane == 15) {
          const float ul = a.u_log ? a.u_log[(long)t * a.Bg + a.b] : wn_uniform(a.seed, t, a.Bg, a.b, 15);
          const double uu = (double)ul;
          gum[cb * 16 + 15] = (float)(log(uu) - log(1.0 - uu));
        }
      }
      if constexpr (TWO_HOP || ONEHOP) {  // skips = the last layer's complete skip slices
        float v = 0.f;
        const bool ok = ww_spin(a.status, lane, [&] {
          const unsigned long long x = ww_get(gin + 256 + tid);  // x granules after the 256 z granules
          v = __uint_as_float((unsigned)x);
          return (unsigned)(x >> 32) == (unsigned)(t + 1);
        });
        if (!ok) flag[0] = 1;
        skv[tid] = fmaxf(v, 0.f);
      } else {  // skips = Σ of the last layer's NC skip partials (running sum and scalings folded in)
        float v[S / WW_THREADS > 0 ? S / WW_THREADS : 1][NC];
        const bool ok = ww_spin(a.status, lane, [&] {
          bool good = true;
#pragma unroll
          for (int r = 0; r < (S + WW_THREADS - 1) / WW_THREADS; ++r) {
            const int j = tid + r * WW_THREADS;
            if (j >= S) continue;
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) {
              const unsigned long long x = ww_get(gin + cc * OUT + j);
              v[r][cc] = __uint_as_float((unsigned)x);
              good = good && (unsigned)(x >> 32) == (unsigned)(t + 1);
            }
          }
          return good;
        });
        if (!ok) flag[0] = 1;
#pragma unroll
        for (int r = 0; r < (S + WW_THREADS - 1) / WW_THREADS; ++r) {
          const int j = tid + r * WW_THREADS;
          if (j >= S) continue;
          float s = 0.f;
#pragma unroll
          for (int cc = 0; cc < NC; ++cc) s += v[r][cc];
          skv[j] = fmaxf(s, 0.f);
        }
      }
      __syncthreads();
      if (flag[0]) return;
      {  // f1 (wavenet.py:840-842)
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const f32x4* xv4 = reinterpret_cast<const f32x4*>(skv + kh * HK);
#pragma unroll
        for (int i4 = 0; i4 < HK / 4; ++i4) {
          const f32x4 xv = xv4[i4];
#pragma unroll
          for (int e = 0; e < 4; ++e) ww_fma4(acc, xv[e], w1[4 * i4 + e]);
        }
        ww_reduce<NKSH>(acc);
        if (kh == 0) {
          f32x4 hv;
          for (int e = 0; e < 4; ++e) hv[e] = fmaxf(acc[e] + b1[e], 0.f);
          reinterpret_cast<f32x4*>(h1)[qh] = hv;
        }
      }
      __syncthreads();
      {  // f2 (wavenet.py:843-844): 8 column quads x 32 row slices, summed on DPP to lane ks = 31
        f32x4 acc = b2;
        if (ks != 0) acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < RK; ++i) ww_fma4(acc, h1[i * 32 + ks], w2[i]);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = sum32_to_lane31(acc[e]);
        if (ks == 31) reinterpret_cast<f32x4*>(lg)[cq] = acc;
      }
      __syncthreads();
      if (wave == 0) {  // sampler (mixture.py:76-107 / gaussian.py:39-52), as k_generate_pipe
        float temp = -INFINITY;
        int idx = lane;
        if (!GAUSS && lane < nr) temp = lg[lane] - gum[cb * 16 + lane];
        argmax16(temp, idx);  // nr <= 10: the mixture logits sit in lanes 0..15
        if (a.logits && lane < a.C) a.logits[((long)a.b * a.T + t) * a.C + lane] = lg[lane];
        if (lane == 0) {
          if (GAUSS) idx = 0;
          const float mean = GAUSS ? lg[0] : lg[nr + idx];
          const float ls = GAUSS ? fmaxf(lg[1], a.log_scale_min_gauss) : fmaxf(lg[2 * nr + idx], a.log_scale_min);
          float x = mean + __expf(ls) * gum[cb * 16 + 15];
          x = fminf(fmaxf(x, -1.f), 1.f);
          const float xn = a.teacher ? a.teacher[(long)a.b * a.T + t] : x;  // wavenet.py:876-878
          if (fuse0) sm[4] = xn;
          else ww_put(sample_gran, (unsigned)(t + 1), xn);
          a.wav[(long)a.b * a.T + t] = x;
          if (a.kout) a.kout[(long)a.b * a.T + t] = idx;
        }
      }
      // unfused: no barrier here -- the next sample's LDS writes (gum[t+1 & 1], skv, h1, lg) each
      // sit behind at least one barrier that wave 0 reaches only after this sampler
      if (fuse0) {
        __syncthreads();
        const float xn = sm[4];
        if (t + 1 < a.T) {
          const float za = base_a + xn * u0a[2], zb = base_b + xn * u0b[2];
          ww_put(a.gran + tid, (unsigned)(t + 2), ww_tanh(za) * ww_sigm(zb));
          ww_put(a.gran + R + tid, (unsigned)(t + 2), xn * fwj + fbj);
        }
        in2 = in1;
        in1 = xn;
      }
    }
    return;
  }

  if constexpr (ONEHOP) {
    ww1_layer<GAUSS>(a, sm, sample_gran);
    return;
  }
  // ============================ layer l, gate-column block c ============================
  const int l = blockIdx.x / NC, c = blockIdx.x % NC;
  float* xin = sm + 16;   // [R] x(t) of this layer
  float* skin = xin + R;  // [S] running skip sum received
  float* z = skin + S;    // [ZC]
  float* zall = z + ZC;   // [R] the layer's whole z (TWO_HOP)
  const int q = tid / NKS, ks = tid % NKS;
  const int q2 = tid / NKS2, ks2 = tid % NKS2;
  const int d = 1 << (l % a.per), Lr = 2 * d + 1;
  long roff = 0;
  for (int l2 = 0; l2 < l; ++l2) roff += (long)NC * (2 * (1 << (l2 % a.per)) + 1) * R;
  float* const ring = a.rings + roff + (long)c * Lr * R;
  for (int i = tid; i < Lr * R; i += WW_THREADS) ring[i] = 0.f;
  f32x4 wt[WW_TAPK], wx[WW_XK], wso[WW_SOK];
  {
    const f32x4* CW = a.conv_w + (long)(l * NC + c) * WW_CK * WW_THREADS + tid;
#pragma unroll
    for (int k = 0; k < WW_TAPK; ++k) wt[k] = CW[(long)k * WW_THREADS];
#pragma unroll
    for (int k = 0; k < WW_XK; ++k) wx[k] = CW[(long)(WW_TAPK + k) * WW_THREADS];
    const f32x4* SW = a.so_w + (long)(l * NC + c) * WW_SOK * WW_THREADS + tid;
#pragma unroll
    for (int k = 0; k < WW_SOK; ++k) wso[k] = SW[(long)k * WW_THREADS];
  }
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const f32x4 cbias = ks == 0 ? reinterpret_cast<const f32x4*>(a.conv_b + (long)l * G + c * GC)[q] : zero4;
  const f32x4 sob = TWO_HOP ? (ks2 == 0 ? reinterpret_cast<const f32x4*>(a.so_b + (long)l * OUT + c * OC)[q2] : zero4)
                            : ((ks2 == 0 && c == 0) ? reinterpret_cast<const f32x4*>(a.so_b + (long)l * OUT)[q2] : zero4);
  const int tap_r0 = ks * WW_TAPK, tap_blk = tap_r0 / R, tap_off = tap_r0 % R;  // blk 0: x(t-2d), 1: x(t-d)
  const unsigned long long* gin = l > 0 ? a.gran + (long)(l - 1) * NG : sample_gran;
  unsigned long long* gout = a.gran + (long)l * NG + c * OUT;
  unsigned long long* const gout_z = a.gran + (long)l * NG;            // TWO_HOP: [NC][ZC] z slices
  unsigned long long* const gout_x = a.gran + (long)l * NG + 256 + c * OC;  // TWO_HOP: this WG's columns
  const float* condp = a.cond + ((long)a.b * a.T) * L * G + (long)l * G + c * GC;
  const bool skip_scale = a.legacy && l > 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int p = 0;  // ring slot of x(t)
  for (int t = 0; t < a.T; ++t) {
    // ---- taps x(t-2d) | x(t-d) of this k-slice, conditioning and bias: before the input arrives ----
    f32x4 acc = zero4;
    {
      const int slot = tap_blk == 0 ? (p + 1 == Lr ? 0 : p + 1) : (p >= d ? p - d : p - d + Lr);
      const float* row = ring + (long)slot * R + tap_off;
#pragma unroll
      for (int i4 = 0; i4 < WW_TAPK / 4; ++i4) {
        const f32x4 xv = ww_ld4(row, i4);
#pragma unroll
        for (int e = 0; e < 4; ++e) ww_fma4(acc, xv[e], wt[4 * i4 + e]);
      }
      if (ks == 0) {
        const f32x4 cd = reinterpret_cast<const f32x4*>(condp + (long)t * L * G)[q];
        for (int e = 0; e < 4; ++e) acc[e] += cbias[e] + cd[e];
      }
    }
    // ---- input x(t) (and the running skip sum) ----
    if (l == 0) {
      if (wave == 0) {  // first_conv 1x1 of the previous sample (wavenet.py:822-826); y_{-1} = 0
        float y = 0.f;
        bool ok = true;
        if (t > 0)
          ok = ww_spin(a.status, lane, [&] {
            const unsigned long long x = ww_get(sample_gran);
            y = __uint_as_float((unsigned)x);
            return (unsigned)(x >> 32) == (unsigned)t;
          });
        if (!ok && lane == 0) flag[0] = 1;
        for (int j = lane; j < R; j += 64) xin[j] = y * a.first_w[j] + a.first_b[j];
      }
    } else if constexpr (TWO_HOP) {
      // x(t) = the out slices of layer l-1 (WGs S/OC..NC-1, granules [256 + S, 256 + OUT)); the running
      // skip of this WG's own skip slice (c < S/OC) = layer l-1's slice c
      const unsigned long long* gx = gin + 256;
      float xv = 0.f, sv = 0.f;
      const bool own_skip = c < S / OC && tid < OC;
      const bool ok = ww_spin(a.status, lane, [&] {
        const unsigned long long x = ww_get(gx + S + tid);
        xv = __uint_as_float((unsigned)x);
        bool good = (unsigned)(x >> 32) == (unsigned)(t + 1);
        if (own_skip) {
          const unsigned long long y = ww_get(gx + c * OC + tid);
          sv = __uint_as_float((unsigned)y);
          good = good && (unsigned)(y >> 32) == (unsigned)(t + 1);
        }
        return good;
      });
      if (!ok) flag[0] = 1;
      xin[tid] = xv;
      if (own_skip) skin[tid] = sv;
    } else {
      constexpr int NR = (OUT + WW_THREADS - 1) / WW_THREADS;
      float v[NR][NC];
      const bool ok = ww_spin(a.status, lane, [&] {
        bool good = true;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int j = tid + r * WW_THREADS;
#pragma unroll
          for (int cc = 0; cc < NC; ++cc) {
            const unsigned long long x = ww_get(gin + cc * OUT + j);
            v[r][cc] = __uint_as_float((unsigned)x);
            good = good && (unsigned)(x >> 32) == (unsigned)(t + 1);
          }
        }
        return good;
      });
      if (!ok) flag[0] = 1;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int j = tid + r * WW_THREADS;  // [skip S | out R] column
        float s = 0.f;
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) s += v[r][cc];
        if (j < S) skin[j] = s;
        else xin[j - S] = s;
      }
    }
    __syncthreads();
    if (flag[0]) return;
    for (int j = tid; j < R; j += WW_THREADS) ring[(long)p * R + j] = xin[j];  // queue append (modules.py:285-288)
    // ---- x(t) rows of the dilated conv (modules.py:291-297), gated activation (:494-510) ----
    {
      const f32x4* xv4 = reinterpret_cast<const f32x4*>(xin + ks * WW_XK);
#pragma unroll
      for (int i4 = 0; i4 < WW_XK / 4; ++i4) {
        const f32x4 xv = xv4[i4];
#pragma unroll
        for (int e = 0; e < 4; ++e) ww_fma4(acc, xv[e], wx[4 * i4 + e]);
      }
    }
    ww_reduce<NKS>(acc);
    if (ks == 0) {
      float2 zz;
      zz.x = ww_tanh(acc[0]) * ww_sigm(acc[2]);
      zz.y = ww_tanh(acc[1]) * ww_sigm(acc[3]);
      reinterpret_cast<float2*>(z)[q] = zz;
    }
    __syncthreads();
    if constexpr (TWO_HOP) {
      // ---- all-gather of the layer's z, then complete skip / out columns of slice c ----
      if (tid < ZC) ww_put(gout_z + c * ZC + tid, (unsigned)(t + 1), z[tid]);
      {
        float zv = 0.f;
        const bool ok = ww_spin(a.status, lane, [&] {
          const unsigned long long x = ww_get(gout_z + tid);
          zv = __uint_as_float((unsigned)x);
          return (unsigned)(x >> 32) == (unsigned)(t + 1);
        });
        if (!ok) flag[0] = 1;
        zall[tid] = zv;
      }
      __syncthreads();
      if (flag[0]) return;
      f32x4 acc2 = zero4;
      const f32x4* zv4 = reinterpret_cast<const f32x4*>(zall + ks2 * WW_SOK);
#pragma unroll
      for (int i4 = 0; i4 < WW_SOK / 4; ++i4) {
        const f32x4 zv = zv4[i4];
#pragma unroll
        for (int e = 0; e < 4; ++e) ww_fma4(acc2, zv[e], wso[4 * i4 + e]);
      }
      ww_reduce<NKS2>(acc2);
      if (ks2 == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lc = 4 * q2 + e, col = c * OC + lc;  // column of [skip S | out R]
          float v = acc2[e] + sob[e];
          if (col < S) {  // skips (wavenet.py:833-836): + running sum of this slice
            if (l > 0) v += skin[lc];
            if (skip_scale) v *= SQH;
          } else {        // residual output
            v += xin[col - S];
            if (a.res_legacy) v *= SQH;
          }
          ww_put(gout_x + lc, (unsigned)(t + 1), v);
        }
      }
    } else {
    // ---- skip / out 1x1 partials of this z slice (modules.py:512-520), published ----
    {
      f32x4 acc2 = zero4;
      const f32x4* zv4 = reinterpret_cast<const f32x4*>(z + ks2 * WW_SOK);
#pragma unroll
      for (int i4 = 0; i4 < WW_SOK / 4; ++i4) {
        const f32x4 zv = zv4[i4];
#pragma unroll
        for (int e = 0; e < 4; ++e) ww_fma4(acc2, zv[e], wso[4 * i4 + e]);
      }
      ww_reduce<NKS2>(acc2);
      if (ks2 == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = 4 * q2 + e;
          float v = acc2[e];
          if (col < S) {  // skips (wavenet.py:833-836)
            if (c == 0) v += sob[e] + (l > 0 ? skin[col] : 0.f);
            if (skip_scale) v *= SQH;
          } else {        // residual output
            if (c == 0) v += sob[e] + xin[col - S];
            if (a.res_legacy) v *= SQH;
          }
          ww_put(gout + col, (unsigned)(t + 1), v);
        }
      }
    }
    }
    p = p + 1 == Lr ? 0 : p + 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the queue append drained before its reads
    __syncthreads();
  }
}

// ======================= R = 256 one-hop layer (k_generate_wide<256, ·, true>) =======================
// The two-hop form all-gathers z inside a layer and then hands complete [skip | out] columns to the
// next layer: two chip-wide hops per layer.  Here the next layer does both halves itself from ONE
// all-gather of the previous layer's (z, x) slices:
//   x_l = rs·(x_{l-1} + O_{l-1}·z_{l-1} + bo_{l-1})              (rs = sqrt(1/2) with legacy residuals)
//   W_x(l)·x_l = rs·W_x(l)·x_{l-1} + [rs·W_x(l)·O_{l-1}]·z_{l-1} + rs·W_x(l)·bo_{l-1}
// so work-group c of layer l holds rs·W_x(l) (its 64 gate columns over 256 x rows), the product
// M = rs·W_x(l)·O_{l-1} (64 gate columns over 256 z rows, formed on the host in float64) and the
// 32 + 32 [out | skip] columns of layer l-1 it completes for the chain (x_l slice c, skip_{l-1}
// slice c) -- 192 weight registers per lane; the tap weights (x(t-2d) | x(t-d), off the serial
// chain) sit in LDS (128 KB).  Per layer and sample the chain is: all-gather (z_{l-1}, x_{l-1}) ->
// gates -> publish (z_l, x_l, skip_{l-1}) slices.  A layer appends x_l(t-1) to its queue from its
// own work-groups' x slices at the start of sample t (off the chain); a tail of NC work-groups
// completes the last layer's skips for the head.  Granules per layer block: [z R | x R | skip R].
template <bool GAUSS>
__device__ void ww1_layer(const WideArgs& a, float* sm, const unsigned long long* sample_gran) {
  constexpr int R = 256, S = 256, G = 512, NC = 8, ZC = 32, GC = 64;
  const float SQH = 0.70710677f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int* flag = reinterpret_cast<int*>(sm);
  const int L = a.L;
  const int l = blockIdx.x / NC, c = blockIdx.x % NC;
  if (l == 0 && a.l0) return;  // layer 0 runs in the head
  const bool tail = l == L;
  f32x4* tapw = reinterpret_cast<f32x4*>(sm + 16);  // [32][256] tap weights
  float* xprev = sm + 16 + 32 * WW_THREADS * 4;      // [R] x_{l-1}(t) (layer 0: x_0(t))
  float* zin = xprev + R;                            // [R] z_{l-1}(t)
  float* sk = zin + R;                               // [32] skip_{l-2}(t), slice c
  const int q = tid >> 4, ks = tid & 15;             // gate / [out | skip] quad, k-slice of 16
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const f32x4* W = a.w1 + (long)(l * NC + c) * W1_NW * WW_THREADS + tid;
  f32x4 wx[16], wm[16], wso[16];
  for (int k = 0; k < 32; ++k) tapw[k * WW_THREADS + tid] = W[(long)k * WW_THREADS];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    wx[k] = W[(long)(32 + k) * WW_THREADS];
    wm[k] = W[(long)(48 + k) * WW_THREADS];
    wso[k] = W[(long)(64 + k) * WW_THREADS];
  }
  const float rs = a.res_legacy ? SQH : 1.f;
  int d = 1, Lr = 3;
  float* ring = nullptr;
  if (!tail) {
    d = 1 << (l % a.per);
    Lr = 2 * d + 1;
    long roff = 0;
    for (int l2 = 0; l2 < l; ++l2) roff += (long)NC * (2 * (1 << (l2 % a.per)) + 1) * R;
    ring = a.rings + roff + (long)c * Lr * R;
    for (int i = tid; i < Lr * R; i += WW_THREADS) ring[i] = 0.f;
  }
  const f32x4 gbias = (ks == 0 && !tail) ? reinterpret_cast<const f32x4*>(a.gb1 + (long)l * G + c * GC)[q] : zero4;
  // [out | skip] column constants of this quad: lc = 4q + e (< 32: out column c·32 + lc, else skip)
  f32x4 sob = zero4;
  if (l > 0 && ks == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int lc = 4 * q + e;
      sob[e] = lc < 32 ? a.so_b[(long)(l - 1) * 2 * R + S + c * 32 + lc] : a.so_b[(long)(l - 1) * 2 * R + c * 32 + lc - 32];
    }
  }
  const int tap_r0 = ks * 32, tap_blk = tap_r0 / R, tap_off = tap_r0 % R;  // blk 0: x(t-2d), 1: x(t-d)
  const unsigned long long* gprev = l > 0 ? a.gran + (long)(l - 1) * W1_GB : nullptr;
  unsigned long long* const gmine = a.gran + (long)l * W1_GB;
  const float* condp = a.cond + ((long)a.b * a.T) * L * G + (long)(tail ? 0 : l) * G + c * GC;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int p = 0, pprev = 0;  // ring slot of x(t), of x(t-1)
  for (int t = 0; t < a.T; ++t) {
    f32x4 acc = zero4;
    if (!tail) {
      if (l > 0 && t > 0) {  // queue append of x_l(t-1): this layer's x slices of sample t-1 (tag t)
        float v = 0.f;
        const bool ok = ww_spin(a.status, lane, [&] {
          const unsigned long long x = ww_get(gmine + R + tid);
          v = __uint_as_float((unsigned)x);
          return (unsigned)(x >> 32) == (unsigned)t;
        });
        if (!ok) flag[0] = 1;
        ring[(long)pprev * R + tid] = v;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (flag[0]) return;
      }
      // ---- taps x(t-2d) | x(t-d) of this k-slice + conditioning + bias: before the input arrives ----
      const int slot = tap_blk == 0 ? (p + 1 == Lr ? 0 : p + 1) : (p >= d ? p - d : p - d + Lr);
      const float* row = ring + (long)slot * R + tap_off;
#pragma unroll
      for (int i4 = 0; i4 < 8; ++i4) {
        const f32x4 xv = ww_ld4(row, i4);
#pragma unroll
        for (int e = 0; e < 4; ++e) ww1_fma4(acc, xv[e], tapw[(4 * i4 + e) * WW_THREADS + tid]);
      }
      if (ks == 0) {
        const f32x4 cd = reinterpret_cast<const f32x4*>(condp + (long)t * L * G)[q];
        for (int e = 0; e < 4; ++e) acc[e] += gbias[e] + cd[e];
      }
    }
    // ---- input ----
    if (l == 0) {
      if (wave == 0) {  // first_conv 1x1 of the previous sample (wavenet.py:822-826); y_{-1} = 0
        float y = 0.f;
        bool ok = true;
        if (t > 0)
          ok = ww_spin(a.status, lane, [&] {
            const unsigned long long x = ww_get(sample_gran);
            y = __uint_as_float((unsigned)x);
            return (unsigned)(x >> 32) == (unsigned)t;
          });
        if (!ok && lane == 0) flag[0] = 1;
        for (int j = lane; j < R; j += 64) xprev[j] = y * a.first_w[j] + a.first_b[j];
      }
      __syncthreads();
      if (flag[0]) return;
      ring[(long)p * R + tid] = xprev[tid];  // queue append of x_0(t) (modules.py:285-288)
    } else {  // the ONE hop: z_{l-1}(t), x_{l-1}(t) (all NC slices) and skip_{l-2}(t) slice c
      float zv = 0.f, xv = 0.f, sv = 0.f;
      const bool want_sk = l >= 2 && tid < 32;
      const bool ok = ww_spin(a.status, lane, [&] {
        const unsigned long long x0 = ww_get(gprev + tid), x1 = ww_get(gprev + R + tid);
        zv = __uint_as_float((unsigned)x0);
        xv = __uint_as_float((unsigned)x1);
        bool good = (unsigned)(x0 >> 32) == (unsigned)(t + 1) && (unsigned)(x1 >> 32) == (unsigned)(t + 1);
        if (want_sk) {
          const unsigned long long x2 = ww_get(gprev + 2 * R + c * 32 + tid);
          sv = __uint_as_float((unsigned)x2);
          good = good && (unsigned)(x2 >> 32) == (unsigned)(t + 1);
        }
        return good;
      });
      if (!ok) flag[0] = 1;
      zin[tid] = zv;
      xprev[tid] = xv;
      if (want_sk) sk[tid] = sv;
      __syncthreads();
      if (flag[0]) return;
      // ---- complete [out | skip] columns of layer l-1 for slice c: x_l slice, skip_{l-1} slice ----
      f32x4 acc2 = zero4;
      const f32x4* zv4 = reinterpret_cast<const f32x4*>(zin + ks * 16);
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const f32x4 z4 = zv4[i4];
#pragma unroll
        for (int e = 0; e < 4; ++e) ww1_fma4(acc2, z4[e], wso[4 * i4 + e]);
      }
      ww_reduce<16>(acc2);
      if (ks == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lc = 4 * q + e;
          if (lc < 32) {  // residual output of layer l-1 = this layer's input slice
            if (!tail) {
              const int j = c * 32 + lc;
              ww_put(gmine + R + j, (unsigned)(t + 1), (xprev[j] + acc2[e] + sob[e]) * rs);
            }
          } else {        // skips (wavenet.py:833-836): + running sum, legacy scaling past layer 0
            const int j = c * 32 + lc - 32;
            float v = acc2[e] + sob[e];
            if (l - 1 > 0) v += sk[lc - 32];
            if (a.legacy && l - 1 > 0) v *= SQH;
            ww_put(gmine + 2 * R + j, (unsigned)(t + 1), v);
          }
        }
      }
    }
    if (!tail) {
      // ---- gates: layer 0 W_x·x_0(t); else rs·W_x·x_{l-1} + M·z_{l-1} (biases folded) ----
      const f32x4* xv4 = reinterpret_cast<const f32x4*>(xprev + ks * 16);
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const f32x4 x4 = xv4[i4];
#pragma unroll
        for (int e = 0; e < 4; ++e) ww1_fma4(acc, x4[e], wx[4 * i4 + e]);
      }
      if (l > 0) {
        const f32x4* zv4 = reinterpret_cast<const f32x4*>(zin + ks * 16);
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const f32x4 z4 = zv4[i4];
#pragma unroll
          for (int e = 0; e < 4; ++e) ww1_fma4(acc, z4[e], wm[4 * i4 + e]);
        }
      }
      ww_reduce<16>(acc);
      if (ks == 0) {
        ww_put(gmine + c * ZC + 2 * q, (unsigned)(t + 1), ww_tanh(acc[0]) * ww_sigm(acc[2]));
        ww_put(gmine + c * ZC + 2 * q + 1, (unsigned)(t + 1), ww_tanh(acc[1]) * ww_sigm(acc[3]));
      }
      if (l == 0 && tid < 32) ww_put(gmine + R + c * 32 + tid, (unsigned)(t + 1), xprev[c * 32 + tid]);
      pprev = p;
      p = p + 1 == Lr ? 0 : p + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // queue appends drained before their reads
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------------- host side

static inline int gate_col_w(int R, int q, int e) { return (e < 2 ? 2 * q + e : R + 2 * q + (e - 2)); }

void ww_pack_conv(const float* conv, int R, int c, std::vector<float>& out) {
  const int NC = ww_nc(R), ZC = R / NC, GC = 2 * ZC, NQ = GC / 4, NKS = WW_THREADS / NQ, G = 2 * R;
  const size_t base = out.size();
  out.resize(base + (size_t)WW_CK * WW_THREADS * 4);
  for (int tid = 0; tid < WW_THREADS; ++tid) {
    const int q = tid / NKS, ks = tid % NKS;
    const int gq = c * NQ + q;  // global gate-permuted quad
    for (int kk = 0; kk < WW_CK; ++kk) {
      // rows of the linearised [3R, G] kernel (taps oldest first): tap rows 32ks.. of [x(t-2d) | x(t-d)],
      // then x(t) rows 2R + 16ks..
      const int row = kk < WW_TAPK ? ks * WW_TAPK + kk : 2 * R + ks * WW_XK + (kk - WW_TAPK);
      for (int e = 0; e < 4; ++e)
        out[base + ((size_t)kk * WW_THREADS + tid) * 4 + e] = conv[(size_t)row * G + gate_col_w(R, gq, e)];
    }
  }
}

void ww_pack_so(const float* skip, const float* outk, int R, int c, std::vector<float>& out) {
  // NC = 2: the partial product of z slice c over all OUT columns; NC = 8 (two-hop): all R z rows
  // for the OUT / NC columns of slice c
  const int NC = ww_nc(R), ZC = R / NC, S = R, OUT = S + R;
  const bool two = NC == 8;
  const int OC = two ? OUT / NC : OUT, NQ2 = OC / 4, NKS2 = WW_THREADS / NQ2;
  const size_t base = out.size();
  out.resize(base + (size_t)WW_SOK * WW_THREADS * 4);
  for (int tid = 0; tid < WW_THREADS; ++tid) {
    const int q2 = tid / NKS2, ks2 = tid % NKS2;
    for (int kk = 0; kk < WW_SOK; ++kk) {
      const int zrow = two ? ks2 * WW_SOK + kk : c * ZC + ks2 * WW_SOK + kk;
      for (int e = 0; e < 4; ++e) {
        const int col = (two ? c * OC : 0) + 4 * q2 + e;
        out[base + ((size_t)kk * WW_THREADS + tid) * 4 + e] =
            col < S ? skip[(size_t)zrow * S + col] : outk[(size_t)zrow * R + (col - S)];
      }
    }
  }
}

size_t ww_ring_floats(int R, int L, int per) {
  size_t n = 0;
  for (int l = 0; l < L; ++l) n += (size_t)ww_nc(R) * (2 * (1 << (l % per)) + 1) * R;
  return n;
}

bool ww_onehop(int R) {
  static const bool on = [] {
    const char* e = std::getenv("TT2_WW_ONEHOP");  // 0: the two-hop R = 256 form
    return !e || std::atoi(e) != 0;
  }();
  return R == 256 && on;
}

size_t ww_lds_bytes(int R, int C) {
  (void)C;
  const int S = R;
  const size_t head = 16 + 2 * S + 32 + 32 + S * 32 + 32 * 32 + 64;
  const size_t layer1 = 16 + 32 * WW_THREADS * 4 + 2 * R + 32;  // one-hop layer: tap weights + x, z, skip
  return sizeof(float) * (ww_onehop(R) ? std::max(head, layer1) : head);
}

int ww_blocks(int R, int L) { return ww_onehop(R) ? (L + 1) * ww_nc(R) + 1 : L * ww_nc(R) + 1; }

const void* ww_kernel(int R, bool gauss) {
  if (R == 128) return gauss ? reinterpret_cast<const void*>(k_generate_wide<128, true>)
                             : reinterpret_cast<const void*>(k_generate_wide<128, false>);
  if (ww_onehop(R))
    return gauss ? reinterpret_cast<const void*>(k_generate_wide<256, true, true>)
                 : reinterpret_cast<const void*>(k_generate_wide<256, false, true>);
  return gauss ? reinterpret_cast<const void*>(k_generate_wide<256, true>)
               : reinterpret_cast<const void*>(k_generate_wide<256, false>);
}

void ww1_pack(const float* conv_l, const float* out_prev, const float* skip_prev, const double* M, float rs, int c,
              std::vector<float>& out) {
  constexpr int R = 256, S = 256, G = 512;
  const size_t base = out.size();
  out.resize(base + (size_t)W1_NW * WW_THREADS * 4, 0.f);
  for (int tid = 0; tid < WW_THREADS; ++tid) {
    const int q = tid >> 4, ks = tid & 15, gq = c * 16 + q;
    auto put = [&](int kk, int e, float v) { out[base + ((size_t)kk * WW_THREADS + tid) * 4 + e] = v; };
    for (int e = 0; e < 4; ++e) {
      const int col = gate_col_w(R, gq, e);
      if (conv_l) {
        for (int kk = 0; kk < 32; ++kk) put(kk, e, conv_l[(size_t)(ks * 32 + kk) * G + col]);
        for (int kk = 0; kk < 16; ++kk) put(32 + kk, e, (out_prev ? rs : 1.f) * conv_l[(size_t)(2 * R + ks * 16 + kk) * G + col]);
        if (M)
          for (int kk = 0; kk < 16; ++kk) put(48 + kk, e, (float)M[(size_t)(ks * 16 + kk) * G + col]);
      }
      if (out_prev) {
        const int lc = 4 * q + e;
        for (int kk = 0; kk < 16; ++kk) {
          const int zrow = ks * 16 + kk;
          put(64 + kk, e, lc < 32 ? out_prev[(size_t)zrow * R + c * 32 + lc] : skip_prev[(size_t)zrow * S + c * 32 + lc - 32]);
        }
      }
    }
  }
}

}  // namespace tt2
