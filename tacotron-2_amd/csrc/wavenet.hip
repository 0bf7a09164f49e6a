// WaveNet MoL vocoder synthesis on MI355X (gfx950).
//
// Reference: code/wavenet_vocoder/models/wavenet.py (incremental :724-911, upsampling :782-803),
// modules.py (CausalConv1D incremental :273-303, ResidualConv1DGLU.step :471-521,
// ConvTranspose2D :736-770), mixture.py (sample_from_discretized_mix_logistic :76-107).
//
// Pipeline per call:
//   1. k_upsample × n_upsample   upsampling network (2D / 1D / Resize / SubPixel / NN) + activation
//   2. gemm                      cond[t][l][·] = c_t·Wc_l + bc_l for ALL t and layers at once
//                                (the conditioning 1×1 never depends on generated samples)
//   3. k_generate                one persistent workgroup per utterance walks t = 0..T-1:
//                                first conv → 24 × (queue taps → dilated conv GEMV → +cond → gated
//                                tanh·σ → skip/out 1×1) → ReLU/1×1/ReLU/1×1 head → MoL sampler.
//      Queues live in LDS as per-layer rings of 2d+1 entries (fast-WaveNet); the next layer's
//      weights are prefetched into registers while the current one is computed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>

#include "common.h"
#include "gemm.h"
#include "wavenet_q.h"
#include "wavenet_wide.h"

namespace tt2 {

static const char* WP = "WaveNet_model/inference/";

// Upsampling network, one launch per layer (wavenet.py:163-203 builds it, :782-803 applies it), on
// channels-first [B][F][T] conditioning (F = cin "frequency" rows).  mode (tt2_wn_config
// upsample_type) and the reference layer each restates:
//   WN_UP_2D        ConvTranspose2D 1->1, kernel (KF, s), stride (1, s), 'same' (modules.py:736-770):
//                   out[f][i*s+j] = Σ_d in[f+pad-d][i] · K[d][j] + b           K [KF][s][1][1]
//   WN_UP_1D        ConvTranspose1D F->F, kernel (1, s), stride (1, s), 'same' (modules.py:697-733):
//                   out[o][i*s+j] = Σ_c in[c][i] · K[0][j][o][c] + b[o]         K [1][s][F][F]
//   WN_UP_RESIZE    nearest-neighbour x s along time, then Conv2D 1->1 kernel (KF, s) 'same'
//                   (modules.py:657-694): out[f][u] = Σ_{d,e} nn[f+d-pf][u+e-pt] · K[d][e] + b
//   WN_UP_SUBPIXEL  Conv2D 1->s kernel (KF, 3) 'same' + periodic shuffle along time
//                   (modules.py:539-654): out[f][w*s+k] = Σ_{d,e} in[f+d-pf][w+e-1] · K[d][e][0][k] + b[k]
//   WN_UP_NN        tf.image.resize NEAREST x hop (modules.py:524-536): out[f][u] = in[f][u/s], no act
// pf = (KF-1)/2, pt = (s-1)/2 (TF 'same': the odd pad goes after).  Activation (upsample_activation):
// none / ReLU / LeakyReLU max(x, alpha·x) (modules.py:23-41).  out_t (nullable) receives the last
// layer transposed to [B][T][F] for the conditioning GEMM.
enum { WN_UP_2D = 0, WN_UP_1D = 1, WN_UP_RESIZE = 2, WN_UP_SUBPIXEL = 3, WN_UP_NN = 4 };
enum { WN_ACT_NONE = 0, WN_ACT_RELU = 1, WN_ACT_LEAKY = 2 };

__global__ void k_upsample(const float* __restrict__ in, float* __restrict__ out, float* __restrict__ out_t,
                           const float* __restrict__ K, const float* __restrict__ bias, int B, int F, int Tin,
                           int s, int KF, int mode, int act, float alpha) {
  const long Tout = (long)Tin * s;
  const long n = (long)B * F * Tout;
  const int pf = (KF - 1) / 2;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int b = e / ((long)F * Tout);
    const long r = e - (long)b * F * Tout;
    const int f = r / Tout;
    const long to = r - (long)f * Tout;
    const int i = to / s, j = to - (long)i * s;
    const float* x = in + (long)b * F * Tin;
    float acc = 0.f;
    if (mode == WN_UP_2D) {
      for (int d = 0; d < KF; ++d) {
        const int ff = f + pf - d;
        if (ff >= 0 && ff < F) acc += x[(long)ff * Tin + i] * K[d * s + j];
      }
      acc += bias[0];
    } else if (mode == WN_UP_1D) {
      const float* kr = K + ((long)j * F + f) * F;
      for (int c = 0; c < F; ++c) acc += x[(long)c * Tin + i] * kr[c];
      acc += bias[f];
    } else if (mode == WN_UP_RESIZE) {
      const int pt = (s - 1) / 2;
      for (int d = 0; d < KF; ++d) {
        const int ff = f + d - pf;
        if (ff < 0 || ff >= F) continue;
        for (int q = 0; q < s; ++q) {
          const long u = to + q - pt;
          if (u >= 0 && u < Tout) acc += x[(long)ff * Tin + u / s] * K[d * s + q];
        }
      }
      acc += bias[0];
    } else if (mode == WN_UP_SUBPIXEL) {
      for (int d = 0; d < KF; ++d) {
        const int ff = f + d - pf;
        if (ff < 0 || ff >= F) continue;
        for (int q = 0; q < 3; ++q) {
          const int w = i + q - 1;
          if (w >= 0 && w < Tin) acc += x[(long)ff * Tin + w] * K[(d * 3 + q) * s + j];
        }
      }
      acc += bias[j];
    } else {  // WN_UP_NN
      acc = x[(long)f * Tin + i];
    }
    const float y = act == WN_ACT_RELU ? fmaxf(acc, 0.f) : (act == WN_ACT_LEAKY ? fmaxf(acc, alpha * acc) : acc);
    out[e] = y;
    if (out_t) out_t[((long)b * Tout + to) * F + f] = y;
  }
}

// WaveNet conditioning from Tacotron mels (wavenet_vocoder/synthesizer.py:56-70 +
// feeder.py:426-428): row b of mels [B][ld_t][F] keeps its first len[b] frames, clipped to
// [lo, hi] (clip_for_wavenet), padded with lo up to T_f, rescaled (x - lo)/(hi - lo) to [0, 1]
// (normalize_for_wavenet) and written channels-first [B][F][T_f], the layout the upsampler
// reads.  32x32 tiles transposed through LDS so both the [t][f] reads and the [f][t] writes
// are coalesced.
__global__ __launch_bounds__(256) void k_cond_from_mels(const float* __restrict__ mels, long ld_t,
                                                        const int* __restrict__ len, int F, int T_f, float lo,
                                                        float hi, int clip, int normalize, float* __restrict__ cond) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, t0 = blockIdx.x * 32, f0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int L = min(len[b], T_f);
  const float scale = normalize ? 1.f / (hi - lo) : 1.f;
  const float off = normalize ? lo : 0.f;
  for (int r = ty; r < 32; r += 8) {
    const int t = t0 + r, f = f0 + tx;
    float v = lo;
    if (t < L && f < F) {
      v = mels[((long)b * ld_t + t) * F + f];
      if (clip) v = fminf(fmaxf(v, lo), hi);
    }
    tile[r][tx] = (v - off) * scale;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int f = f0 + r, t = t0 + tx;
    if (f < F && t < T_f) cond[((long)b * F + f) * T_f + t] = tile[tx][r];
  }
}

// Column order of the gated conv / cond outputs per quad q: {a_2q, a_2q+1, b_2q, b_2q+1}
// so the lane that reduces quad q can apply tanh(a)·σ(b) without a cross-lane exchange.
static inline int gate_col(int R, int q, int e) { return (e < 2 ? 2 * q + e : R + 2 * q + (e - 2)); }

// ---------------------------------------------------------------------------------------------
// Layer-pipelined generator.  Generation is a strict serial chain (sample t+1 needs the sample
// drawn from all 24 layers of sample t), so its speed is the latency of one pass through the
// stack.  One CU cannot hold the 3.1 MB of per-sample weights, and streaming them from L2 every
// sample is what bounds a single-CU generator (~43 GB/s per CU -> 75 us/sample).  Here the stack is
// cut into NST = ceil(L/3) stages of three layers; each stage is one 512-thread workgroup on its
// own CU that keeps its layers' weights in REGISTERS (64 VGPRs per layer per lane) and its layers'
// fast-WaveNet queues in LDS for the whole utterance.  Per sample the activations travel
// stage -> stage as 128 data-tagged 8-byte granules {tag = t+1, fp32 bits} (x and the running skip
// sum) written with relaxed agent-scope atomic stores and swept by one wave of the consumer
// (cdna_hip_programming.md §6 Guideline 16, R2: the data is the flag, no fences); the last stage
// runs the ReLU/1x1/ReLU/1x1 head and the MoL sampler and hands the sample back to stage 0.
// Every spin is bounded (status word + early exit), every polled word is zeroed before the launch.
// Stage s of utterance u runs as block ((u/8)*NST + s)*8 + u%8: with round-robin dispatch all
// stages of one utterance share an XCD (speed only; the protocol is placement-independent).
// ---------------------------------------------------------------------------------------------
constexpr int WN_THREADS = 256;   // 4 waves, 1 per SIMD: 512 registers per lane (VGPR + AGPR)
constexpr int WN_LPS = 3;         // layers per stage
constexpr int WN_TK = 16;         // conv tap rows per k-slice (128 / 8): x(t-2d) | x(t-d)
constexpr int WN_XK = 8;          // conv x(t) rows per k-slice (64 / 8)
constexpr int WN_CK = WN_TK + WN_XK;
constexpr int WN_SK = 8;          // skip/out rows per k-slice (64 / 8)
constexpr int WN_GR = 128;        // granules per stage edge (x[64] | skip[64])

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;

struct GenArgs {
  int B, T, L, per, nst;   // utterances in this launch, samples, layers, layers per stack, stages
  int b0, Bg;              // first global utterance of this launch, global batch
  const float* first_w; const float* first_b;  // [R], [R]
  const f32x4* conv_w;  // [L][12][512] float4: tid = q*16+ks holds rows 12ks.. of quad q
  const float* conv_b;  // [L][G] gate-permuted
  const float* cond;    // [Bg][T][L][G] gate-permuted (includes the cin_conv bias)
  const f32x4* so_w;    // [L][4][512] float4: rows 4ks.. of [Ws|Wo] quad q
  const float* so_b;    // [L][2R] = [bs | bo]
  const float* f1_w; const float* f1_b;  // [S][S], [S]
  const float* f2_w; const float* f2_b;  // [S][C], [C]
  int C;
  int legacy, res_legacy;
  float log_scale_min, log_scale_min_gauss;
  const float* u_mix; const float* u_log;  // [T][Bg][nr], [T][Bg] or null (Gaussian: u_log = N(0,1) draws)
  uint64_t seed;
  const float* teacher;  // [Bg][T] or null
  float* wav; int* kout; float* logits;    // [Bg][T], [Bg][T], [Bg][T][C]
  unsigned long long* gran;  // [B][nst][128]
  int* status;               // 0 ok, else spin timeout code
  long long* stamps;         // [64][8] s_memrealtime stamps of utterance 0 at sample T/2 (diagnostic)
};

__device__ __forceinline__ float gumbel_L(double u) { return (float)log(-log(u)); }

// keeps a loop-invariant per-lane offset from being hoisted (and then spilled) out of the sample loop
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned tag, float v) {
  __hip_atomic_store((gu64*)g, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// One wave: sweep n (<= 128) granules until every tag == tag.  Lane i returns granules i, i+64.
// Bounded: gives up after ~4 s (or when another stage reported a failure) and returns false.
__device__ bool sweep(const unsigned long long* g, int n, unsigned tag, float& v0, float& v1, int* status,
                      int lane) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  for (unsigned it = 0;; ++it) {
    bool ok = true;
    if (lane < n) {
      const unsigned long long x = __hip_atomic_load((gu64*)(g + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v0 = __uint_as_float((unsigned)x);
      ok = (unsigned)(x >> 32) == tag;
    }
    if (lane + 64 < n) {
      const unsigned long long x =
          __hip_atomic_load((gu64*)(g + lane + 64), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v1 = __uint_as_float((unsigned)x);
      ok = ok && (unsigned)(x >> 32) == tag;
    }
    if (__all(ok)) return true;
    if ((it & 255) == 255) {
      const int st = __hip_atomic_load((gi32*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (st != 0) return false;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
        if (lane == 0) __hip_atomic_store((gi32*)status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
}

// 256 threads: tid = q*8 + ks, q = column quad (32 x 4 gate columns / 32 x 4 skip|out columns),
// ks = k-slice (8).  Per lane and layer: 16 float4 of tap weights (used off the critical path;
// the allocator parks them in AGPRs), 8 float4 of x(t) conv weights and 8 float4 of skip/out
// weights (VGPRs).  Cross-slice sums are 3-level DPP reductions inside 8-lane groups.
__device__ __forceinline__ void sum8x4(f32x4& a) {
#define TT2_STEP(C)                                                                                  \
  {                                                                                                  \
    const float t0 = dpp_f<C>(a[0]), t1 = dpp_f<C>(a[1]), t2 = dpp_f<C>(a[2]), t3 = dpp_f<C>(a[3]); \
    a[0] += t0; a[1] += t1; a[2] += t2; a[3] += t3;                                                  \
  }
  TT2_STEP(DPP_XOR1) TT2_STEP(DPP_XOR2) TT2_STEP(DPP_HALF_MIRROR)
#undef TT2_STEP
}

// acc += x·w on four columns: WN_PK = 1 issues two v_pk_fma_f32 (x broadcast by op_sel_hi) instead
// of four v_fma_f32 (A/B switch for the per-layer chain products)
#ifndef WN_PK
#define WN_PK 0
#endif
typedef float wn_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void wn_fma4(f32x4& acc, float x, const f32x4& w) {
  if (WN_PK) {
    const wn_f32x2 xx = {x, x};
    const wn_f32x2 lo = __builtin_elementwise_fma(xx, wn_f32x2{w[0], w[1]}, wn_f32x2{acc[0], acc[1]});
    const wn_f32x2 hi = __builtin_elementwise_fma(xx, wn_f32x2{w[2], w[3]}, wn_f32x2{acc[2], acc[3]});
    acc = f32x4{lo[0], lo[1], hi[0], hi[1]};
  } else {
    acc[0] += x * w[0]; acc[1] += x * w[1]; acc[2] += x * w[2]; acc[3] += x * w[3];
  }
}

// Explicit AGPR residency for the off-critical-path tap weights (the allocator otherwise parks the
// critical-path weights there and pays a v_accvgpr_read per use inside the serial chain).
__device__ __forceinline__ float agpr_put(float v) {
  float r;
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(r) : "v"(v));
  return r;
}
__device__ __forceinline__ float agpr_get(float r) {
  float v;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(r));
  return v;
}

// GAUSS: out_channels == 2 Gaussian head (a template parameter so the MoL instantiation keeps
// its register allocation: a runtime flag costs the register-resident generator spills)
template <bool LEGACY, bool RES_LEGACY, bool GAUSS>
__global__ __launch_bounds__(WN_THREADS, 1) void k_generate_pipe(GenArgs a) {
  constexpr int R = 64, G = 128, S = 64, NT = WN_THREADS;
  const int blk = blockIdx.x, xl = blk & 7, grp = blk >> 3;
  const int s = grp % a.nst, bl = (grp / a.nst) * 8 + xl;
  if (bl >= a.B) return;
  const int b = a.b0 + bl;  // global utterance
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = tid >> 3, ks = tid & 7;
  const int L = a.L, per = a.per, l0 = s * WN_LPS, nl = min(WN_LPS, L - l0);
  const bool first = s == 0, last = s + 1 == a.nst;
  unsigned long long* gin = a.gran + ((long)bl * a.nst + (first ? a.nst - 1 : s - 1)) * WN_GR;
  unsigned long long* gout = a.gran + ((long)bl * a.nst + s) * WN_GR;

  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xcur = sm;                  // [64] input x(t) of the layer being computed
  float* z = xcur + R;               // [64]
  float* fwb = z + R;                // [128] first_conv weight | bias (stage 0)
  float* skr = fwb + 2 * R;          // [64] received skip sum
  float* skv = skr + S;              // [64]
  float* h1 = skv + S;               // [64]
  float* lg = h1 + S;                // [32]
  float* gum = lg + 32;              // [2][16] Gumbel terms (+ [15] = logistic noise) by t&1
  float* cbuf = gum + 32;            // [2][3*128] conditioning by t&1
  float* cbias = cbuf + 2 * WN_LPS * G;  // [3*128]
  float* sbias = cbias + WN_LPS * G;     // [3*128]
  float* hw1 = sbias + WN_LPS * G;       // [64*64]
  float* hw2 = hw1 + S * S;              // [64*32]
  float* hb = hw2 + S * 32;              // [64 + 32]
  int* flag = reinterpret_cast<int*>(hb + 96);  // [4] abort
  float* rings = hb + 100;                      // this stage's queues

  // ---- per-stage layer geometry (wave-uniform) ----
  int dl[WN_LPS], Ll[WN_LPS], ro[WN_LPS], pos[WN_LPS];  // pos[j] = t mod L_j, kept incrementally
  {
    int off = 0;
#pragma unroll
    for (int j = 0; j < WN_LPS; ++j) {
      dl[j] = 1 << ((l0 + j) % per);
      Ll[j] = 2 * dl[j] + 1;
      ro[j] = off;
      pos[j] = 0;
      off += (j < nl) ? Ll[j] * R : 0;
    }
    for (int i = tid; i < off; i += NT) rings[i] = 0.f;
  }
  // ---- weights for the whole utterance, in registers ----
  float wt[WN_LPS][WN_TK * 4];  // AGPRs
  f32x4 wx[WN_LPS][WN_XK], wsr[WN_LPS][WN_SK];
#pragma unroll
  for (int j = 0; j < WN_LPS; ++j) {
    const int l = min(l0 + j, L - 1);
#pragma unroll
    for (int kk = 0; kk < WN_TK; ++kk) {
      const f32x4 w = a.conv_w[((long)l * WN_CK + kk) * NT + tid];
#pragma unroll
      for (int e = 0; e < 4; ++e) wt[j][4 * kk + e] = agpr_put(w[e]);
    }
#pragma unroll
    for (int kk = 0; kk < WN_XK; ++kk) wx[j][kk] = a.conv_w[((long)l * WN_CK + WN_TK + kk) * NT + tid];
#pragma unroll
    for (int kk = 0; kk < WN_SK; ++kk) wsr[j][kk] = a.so_w[((long)l * WN_SK + kk) * NT + tid];
  }
  for (int i = tid; i < nl * G; i += NT) {
    cbias[i] = a.conv_b[(long)l0 * G + i];
    sbias[i] = a.so_b[(long)l0 * 2 * R + i];
  }
  if (last) {
    for (int i = tid; i < S * S; i += NT) hw1[i] = a.f1_w[i];
    for (int i = tid; i < S * 32; i += NT) {
      const int k = i >> 5, c = i & 31;
      hw2[i] = c < a.C ? a.f2_w[k * a.C + c] : 0.f;
    }
    for (int i = tid; i < 96; i += NT) hb[i] = i < S ? a.f1_b[i] : (i - S < a.C ? a.f2_b[i - S] : 0.f);
  }
  const f32x4* cond4 = reinterpret_cast<const f32x4*>(a.cond);
  const long crow = (long)L * G / 4;  // float4 per sample row
  if (tid < nl * G / 4) reinterpret_cast<f32x4*>(cbuf)[tid] = cond4[((long)b * a.T) * crow + l0 * G / 4 + tid];
  if (first && tid < R) { fwb[tid] = a.first_w[tid]; fwb[R + tid] = a.first_b[tid]; }
  if (tid == 0) flag[0] = 0;
  const float SQH = 0.70710677f;  // float32(np.sqrt(0.5))
  const int nr = a.C / 3;
  f32x4 skips = {0.f, 0.f, 0.f, 0.f}, xres = {0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  for (int t = 0; t < a.T; ++t) {
    const int cb_cur = t & 1;
    // ---- off the critical path (overlaps the hand-off wait) ----
    f32x4 cn = {0.f, 0.f, 0.f, 0.f};
    const bool has_next = t + 1 < a.T;
    if (has_next && tid < nl * G / 4) cn = cond4[((long)b * a.T + t + 1) * crow + l0 * G / 4 + tid];
    if (GAUSS && last && wave == 1) {  // this sample's N(0,1) draw (injected in u_log, or Box-Muller)
      if (lane == 15) {
        float nz;
        if (a.u_log) {
          nz = a.u_log[(long)t * a.Bg + b];
        } else {
          nz = wn_gauss(a.seed, t, a.Bg, b);
        }
        gum[cb_cur * 16 + 15] = nz;
      }
    } else if (!GAUSS && last && wave == 1) {  // this sample's Gumbel terms and logistic noise
      if (lane < nr) {
        const float um = a.u_mix ? a.u_mix[((long)t * a.Bg + b) * nr + lane]
                                 : wn_uniform(a.seed, t, a.Bg, b, lane);
        gum[cb_cur * 16 + lane] = gumbel_L((double)um);
      } else if (lane == 15) {
        const float ul = a.u_log ? a.u_log[(long)t * a.Bg + b]
                                 : wn_uniform(a.seed, t, a.Bg, b, 15);
        const double uu = (double)ul;
        gum[cb_cur * 16 + 15] = (float)(log(uu) - log(1.0 - uu));
      }
    }
    // dilated-conv taps x(t-2d), x(t-d) of every layer of this stage are already in the queues:
    // their part of the conv (2/3 of its rows), the conv bias and the conditioning are summed now
    f32x4 tp[WN_LPS];
#pragma unroll
    for (int j = 0; j < WN_LPS; ++j) {
      tp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j >= nl) continue;
      const int p = pos[j], Lj = Ll[j];
      const int slot = ks < 4 ? (p + 1 == Lj ? 0 : p + 1)                               // x(t-2d)
                              : (p + dl[j] + 1 >= Lj ? p + dl[j] + 1 - Lj : p + dl[j] + 1);  // x(t-d)
      const f32x4* tv = reinterpret_cast<const f32x4*>(rings + ro[j] + slot * R + 16 * (ks & 3));
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const f32x4 xv = tv[k4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * (4 * k4 + e);
          const float w0 = agpr_get(wt[j][r]), w1 = agpr_get(wt[j][r + 1]);
          const float w2 = agpr_get(wt[j][r + 2]), w3 = agpr_get(wt[j][r + 3]);
          acc[0] += xv[e] * w0; acc[1] += xv[e] * w1; acc[2] += xv[e] * w2; acc[3] += xv[e] * w3;
        }
      }
      if (ks == 0) {
        const f32x4 cb = reinterpret_cast<const f32x4*>(cbias + j * G)[q];
        const f32x4 cd = reinterpret_cast<const f32x4*>(cbuf + cb_cur * WN_LPS * G + j * G)[q];
        for (int e = 0; e < 4; ++e) acc[e] += cb[e] + cd[e];
      }
      tp[j] = acc;
    }
    // ---- receive this stage's input (wave 0 sweeps; one barrier publishes it to the stage) ----
    if (wave == 0) {
      float v0 = 0.f, v1 = 0.f;
      bool ok = true;
      if (first) {
        if (t > 0) ok = sweep(gin, 1, (unsigned)t, v0, v1, a.status, lane);
        const float xp = __shfl(v0, 0);
        v0 = xp * fwb[lane] + fwb[R + lane];  // first_conv 1x1 (wavenet.py:822): x0 = y_{t-1}·w + b
      } else {
        ok = sweep(gin, WN_GR, (unsigned)(t + 1), v0, v1, a.status, lane);
      }
      if (a.stamps && lane == 0 && bl == 0 && a.b0 == 0 && t == a.T / 2)
        a.stamps[s * 8 + 7] = __builtin_amdgcn_s_memrealtime();
      if (!ok) {
        if (lane == 0) flag[0] = 1;
      } else {
        xcur[lane] = v0;
        rings[ro[0] + pos[0] * R + lane] = v0;
        skr[lane] = v1;
      }
    }
    __syncthreads();
    if (flag[0]) return;
    const bool stamp = a.stamps && bl == 0 && a.b0 == 0 && t == a.T / 2 && tid == 0 && s < 64;
    if (stamp) a.stamps[s * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    if (stamp) a.stamps[448 + 2 * s] = __builtin_amdgcn_s_memtime();
    if (ks == 0) {
      if (q < 16) {
        if (!first) skips = reinterpret_cast<const f32x4*>(skr)[q];
      } else {
        xres = reinterpret_cast<const f32x4*>(xcur)[q - 16];
      }
    }

#pragma unroll
    for (int j = 0; j < WN_LPS; ++j) {
      if (j >= nl) break;
      const int l = l0 + j;
      // conv rows of x(t) (modules.py:283-297) on top of the precomputed tap part
      f32x4 acc = tp[j];
      {
        float xv[8];
        {
          const f32x4* xv4 = reinterpret_cast<const f32x4*>(xcur + 8 * ks);
          const f32x4 x0 = xv4[0], x1 = xv4[1];
          for (int e = 0; e < 4; ++e) { xv[e] = x0[e]; xv[4 + e] = x1[e]; }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          wn_fma4(acc, xv[i], wx[j][i]);
        }
      }
      const f32x4 sb = reinterpret_cast<const f32x4*>(sbias + j * G)[q];  // for the skip/out phase
      sum8x4(acc);
      if (ks == 0) {  // tanh(a)·σ(b) (modules.py:494-510)
        float2 zz;
        zz.x = tanh_rcp(acc[0]) * sigm_fast(acc[2]);
        zz.y = tanh_rcp(acc[1]) * sigm_fast(acc[3]);
        reinterpret_cast<float2*>(z)[q] = zz;
      }
      // next sample's conditioning -> the other cbuf half: its last reader was the previous
      // sample's tap precompute, and the barrier closing this layer orders it before the next one
      if (j == 0 && has_next && tid < nl * G / 4) reinterpret_cast<f32x4*>(cbuf + (cb_cur ^ 1) * WN_LPS * G)[tid] = cn;
      __syncthreads();
      // skip / out 1x1 (modules.py:512-520): 8 rows x 4 columns of [Ws | Wo] per lane
      f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};
      {
        const f32x4* zv4 = reinterpret_cast<const f32x4*>(z + 8 * ks);
#pragma unroll
        for (int k4 = 0; k4 < 2; ++k4) {
          const f32x4 zv = zv4[k4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            wn_fma4(acc2, zv[e], wsr[j][4 * k4 + e]);
          }
        }
      }
      sum8x4(acc2);
      if (ks == 0) {
        if (q < 16) {  // skip sum (wavenet.py:833-836)
          f32x4 sv;
          for (int e = 0; e < 4; ++e) sv[e] = acc2[e] + sb[e];
          if (l == 0) skips = sv;
          else if (LEGACY) for (int e = 0; e < 4; ++e) skips[e] = (skips[e] + sv[e]) * SQH;
          else for (int e = 0; e < 4; ++e) skips[e] = skips[e] + sv[e];
          if (j + 1 == nl && !last) {
            const int go = opaque(R + 4 * q);
            for (int e = 0; e < 4; ++e) put_granule(gout + go + e, (unsigned)(t + 1), skips[e]);
            if (a.stamps && tid == 0 && bl == 0 && a.b0 == 0 && t == a.T / 2)
              a.stamps[s * 8 + 6] = __builtin_amdgcn_s_memrealtime();
          }
        } else if (l + 1 < L) {  // residual output (modules.py:517-520)
          const int c4 = opaque(q - 16);  // channel quad
          for (int e = 0; e < 4; ++e) {
            xres[e] = (acc2[e] + sb[e]) + xres[e];
            if (RES_LEGACY) xres[e] = xres[e] * SQH;
          }
          if (j + 1 < nl) {  // next layer of this stage: its x(t) and its queue
            const int jn = j + 1 < WN_LPS ? j + 1 : 0;
            reinterpret_cast<f32x4*>(xcur)[c4] = xres;
            reinterpret_cast<f32x4*>(rings + ro[jn] + pos[jn] * R)[c4] = xres;
          } else {
            for (int e = 0; e < 4; ++e) put_granule(gout + 4 * c4 + e, (unsigned)(t + 1), xres[e]);
          }
        }
      }
      __syncthreads();
      if (stamp) a.stamps[s * 8 + 1 + j] = __builtin_amdgcn_s_memrealtime();
      if (stamp && j + 1 == nl) a.stamps[448 + 2 * s + 1] = __builtin_amdgcn_s_memtime();
    }
#pragma unroll
    for (int j = 0; j < WN_LPS; ++j) pos[j] = pos[j] + 1 == Ll[j] ? 0 : pos[j] + 1;
    if (!last) continue;

    // ---- head: ReLU -> 1x1 (S->S) -> ReLU -> 1x1 (S->C) (wavenet.py:840-844) and the MoL
    //      sampler (mixture.py:76-107), all in wave 0 after one barrier ----
    if (ks == 0 && q < 16)
      for (int e = 0; e < 4; ++e) skv[4 * q + e] = fmaxf(skips[e], 0.f);
    __syncthreads();
    if (wave != 0) continue;
    {  // f1: 16 column quads x 4 slices of 16 rows per lane
      const int q2 = lane >> 2, k2 = lane & 3;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const f32x4* xv4 = reinterpret_cast<const f32x4*>(skv + 16 * k2);
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const f32x4 xv = xv4[k4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x4 w = reinterpret_cast<const f32x4*>(hw1 + (16 * k2 + 4 * k4 + e) * S)[q2];
          acc[0] += xv[e] * w[0]; acc[1] += xv[e] * w[1]; acc[2] += xv[e] * w[2]; acc[3] += xv[e] * w[3];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[e] += dpp_f<DPP_XOR1>(acc[e]);
        acc[e] += dpp_f<DPP_XOR2>(acc[e]);
      }
      if (k2 == 0) {
        const f32x4 bb = reinterpret_cast<const f32x4*>(hb)[q2];
        f32x4 hv;
        for (int e = 0; e < 4; ++e) hv[e] = fmaxf(acc[e] + bb[e], 0.f);
        reinterpret_cast<f32x4*>(h1)[q2] = hv;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's h1 stores before its loads
    {  // f2: 8 column quads (32 >= C) x 8 slices of 8 rows per lane
      const int q3 = lane >> 3, k3 = lane & 7;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const f32x4* xv4 = reinterpret_cast<const f32x4*>(h1 + 8 * k3);
#pragma unroll
      for (int k4 = 0; k4 < 2; ++k4) {
        const f32x4 xv = xv4[k4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x4 w = reinterpret_cast<const f32x4*>(hw2 + (8 * k3 + 4 * k4 + e) * 32)[q3];
          acc[0] += xv[e] * w[0]; acc[1] += xv[e] * w[1]; acc[2] += xv[e] * w[2]; acc[3] += xv[e] * w[3];
        }
      }
      sum8x4(acc);
      if (k3 == 0) {
        const f32x4 bb = reinterpret_cast<const f32x4*>(hb + S)[q3];
        f32x4 lv;
        for (int e = 0; e < 4; ++e) lv[e] = acc[e] + bb[e];
        reinterpret_cast<f32x4*>(lg)[q3] = lv;
        if (a.logits)
          for (int e = 0; e < 4; ++e)
            if (4 * q3 + e < a.C) a.logits[((long)b * a.T + t) * a.C + 4 * q3 + e] = lv[e];
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    if (stamp) a.stamps[s * 8 + 4] = __builtin_amdgcn_s_memrealtime();
    {
      float temp = -INFINITY;
      int idx = lane;
      if (!GAUSS && lane < nr) temp = lg[lane] - gum[cb_cur * 16 + lane];
      argmax16(temp, idx);  // nr <= 10: the mixture logits sit in lanes 0..15
      if (lane == 0) {
        // MoL: mixture idx (mixture.py:92-105); Gaussian: out = [mean, log_scale] (gaussian.py:39-52)
        if (GAUSS) idx = 0;
        const float mean = GAUSS ? lg[0] : lg[nr + idx];
        const float ls = GAUSS ? fmaxf(lg[1], a.log_scale_min_gauss) : fmaxf(lg[2 * nr + idx], a.log_scale_min);
        float x = mean + expf(ls) * gum[cb_cur * 16 + 15];
        x = fminf(fmaxf(x, -1.f), 1.f);
        const float xn = a.teacher ? a.teacher[(long)b * a.T + t] : x;  // wavenet.py:876-878
        put_granule(gout, (unsigned)(t + 1), xn);
        if (stamp) a.stamps[s * 8 + 5] = __builtin_amdgcn_s_memrealtime();
        a.wav[(long)b * a.T + t] = x;
        if (a.kout) a.kout[(long)b * a.T + t] = idx;
      }
    }
  }
}

// Standalone MoL sampler: one wave per row.
__global__ void k_mol_sample(const float* __restrict__ logits, const float* __restrict__ u_mix,
                             const float* __restrict__ u_log, int n, int nr, float lsm, float* __restrict__ x,
                             int* __restrict__ k) {
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const float* lg = logits + (long)row * 3 * nr;
  float temp = -INFINITY;
  int idx = lane;
  if (lane < nr) temp = lg[lane] - gumbel_L((double)u_mix[(long)row * nr + lane]);
  for (int o = 32; o > 0; o >>= 1) {
    const float ot = __shfl_xor(temp, o);
    const int oi = __shfl_xor(idx, o);
    if (ot > temp || (ot == temp && oi < idx)) { temp = ot; idx = oi; }
  }
  if (lane == 0) {
    const float mean = lg[nr + idx];
    const float ls = fmaxf(lg[2 * nr + idx], lsm);
    const double uu = (double)u_log[row];
    const float noise = (float)(log(uu) - log(1.0 - uu));
    float v = mean + expf(ls) * noise;
    x[row] = fminf(fmaxf(v, -1.f), 1.f);
    k[row] = idx;
  }
}

}  // namespace tt2

struct tt2_wn_ctx {
  tt2_wn_config cfg;
  int dev = 0;
  hipStream_t stream = nullptr;
  tt2::WeightMap host;
  bool finalized = false;
  int R, G, S, L, C, cin;
  long hop;
  tt2::DevBuf first_w, first_b, conv_w, conv_b, cond_w, cond_b, so_w, so_b, f1_w, f1_b, f2_w, f2_b;
  tt2::DevBuf w1, gb1, l0;  // R = 256 one-hop form (wavenet_wide.h WideArgs::w1 / gb1 / l0)
  tt2::DevBuf up_k[8], up_b[8];
  tt2::DevBuf cin_d, up_a, up_b_buf, c_up_t, cond, umix, ulog, teacher, wav, kout, logits, gran, stamps;
  int chunk = 1;                 // utterances per generation launch
  bool wide = false;             // R = 128 / 256: k_generate_wide (wavenet_wide.hip), one utterance per launch
  tt2::DevBuf rings;             // k_generate_wide's per-work-group fast-WaveNet queues
  int* status_host = nullptr;    // pinned: spin-timeout word of the last launch
  tt2::DevBuf gcv;               // [gc_B][L][G] gate-permuted global-condition terms (set_global_condition)
  int gc_B = 0;
  bool quantize = false;         // input_type 'mulaw-quantize': k_generate_q (wavenet_q.hip), natural layouts
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool timed = false;
};

namespace tt2 {

// cond[b][t][:] += gcv[b][:]: the per-row, time-invariant global-condition term of every layer
__global__ void k_add_gc(float* __restrict__ cond, const float* __restrict__ gcv, int B, long T, int LG) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * T * LG) return;
  const int n = (int)(i % LG);
  const int b = (int)(i / ((long)T * LG));
  cond[i] += gcv[(long)b * LG + n];
}

static void wupload(DevBuf& d, const std::vector<float>& h) {
  d.alloc(h.size() * sizeof(float));
  TT2_HIP(hipMemcpy(d.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
}

// upsampling-network weights (local conditioning on)
static void wn_upload_upsampler(tt2_wn_ctx* c) {
  const WeightMap& wm = c->host;
  const std::string P(WP);
  const int cin = c->cin;
  static const char* kUpName[4] = {"ConvTranspose2D_layer_", "ConvTranspose1D_layer_", "ResizeConvolution_layer_",
                                   "SubPixelConvolution_layer_"};
  const int ut = c->cfg.upsample_type;
  for (int i = 0; cin > 0 && ut != WN_UP_NN && i < c->cfg.n_upsample; ++i) {
    const std::string sc = P + "local_conditioning_upsampling_" + std::to_string(i + 1) + "/" + kUpName[ut] +
                           std::to_string(i) + "/";
    const int s = c->cfg.upsample_scales[i], kf = c->cfg.freq_axis_kernel_size;
    if (ut == WN_UP_1D) {
      wupload(c->up_k[i], need(wm, sc + "kernel", {1, s, cin, cin}).data);
      wupload(c->up_b[i], need(wm, sc + "bias", {cin}).data);
    } else if (ut == WN_UP_SUBPIXEL) {
      std::vector<float> k = need(wm, sc + "kernel", {kf, 3, 1, s}).data;
      if (!c->cfg.NN_init)  // SubPixelConvolution.build (modules.py:585-593): every channel = channel 0
        for (int q = 0; q < kf * 3; ++q)
          for (int o = 1; o < s; ++o) k[(size_t)q * s + o] = k[(size_t)q * s];
      wupload(c->up_k[i], k);
      wupload(c->up_b[i], need(wm, sc + "bias", {s}).data);
    } else {
      wupload(c->up_k[i], need(wm, sc + "kernel", {kf, s, 1, 1}).data);
      wupload(c->up_b[i], need(wm, sc + "bias", {1}).data);
    }
  }
}

// 'mulaw-quantize' (k_generate_q): natural column orders -- the first conv [Q][R], the dilated
// convs [L][3R][G], [skip | out] [L][R][S + R], the conditioning 1x1s [cin][L][G]
static void wn_finalize_q(tt2_wn_ctx* c) {
  const WeightMap& wm = c->host;
  const std::string P(WP);
  const int R = c->R, G = c->G, S = c->S, L = c->L, Q = c->C, cin = c->cin, kw = c->cfg.kernel_size;
  TT2_HIP(hipSetDevice(c->dev));
  wupload(c->first_w, need(wm, P + "input_convolution/kernel", {1, Q, R}).data);
  wupload(c->first_b, need(wm, P + "input_convolution/bias", {R}).data);
  std::vector<float> cw((size_t)L * kw * R * G), cb((size_t)L * G), sow((size_t)L * R * (S + R)), sob((size_t)L * (S + R));
  std::vector<float> condw((size_t)std::max(cin, 1) * L * G, 0.f), condb((size_t)L * G, 0.f);
  for (int l = 0; l < L; ++l) {
    const std::string s = P + "ResidualConv1DGLU_" + std::to_string(l) + "/";
    const std::string ln = "_ResidualConv1DGLU_" + std::to_string(l) + "/";
    const auto& k = need(wm, s + "residual_block_causal_conv" + ln + "kernel", {kw, R, G});
    const auto& bb = need(wm, s + "residual_block_causal_conv" + ln + "bias", {G});
    const auto& ksk = need(wm, s + "residual_block_skip_conv" + ln + "kernel", {1, G / 2, S});
    const auto& bsk = need(wm, s + "residual_block_skip_conv" + ln + "bias", {S});
    const auto& ko = need(wm, s + "residual_block_out_conv" + ln + "kernel", {1, G / 2, R});
    const auto& bo = need(wm, s + "residual_block_out_conv" + ln + "bias", {R});
    std::copy(k.data.begin(), k.data.end(), cw.begin() + (size_t)l * kw * R * G);
    std::copy(bb.data.begin(), bb.data.end(), cb.begin() + (size_t)l * G);
    for (int j = 0; j < R; ++j) {
      for (int o = 0; o < S; ++o) sow[((size_t)l * R + j) * (S + R) + o] = ksk.data[(size_t)j * S + o];
      for (int o = 0; o < R; ++o) sow[((size_t)l * R + j) * (S + R) + S + o] = ko.data[(size_t)j * R + o];
    }
    for (int o = 0; o < S; ++o) sob[(size_t)l * (S + R) + o] = bsk.data[o];
    for (int o = 0; o < R; ++o) sob[(size_t)l * (S + R) + S + o] = bo.data[o];
    if (cin > 0) {
      const auto& kc = need(wm, s + "residual_block_cin_conv" + ln + "kernel", {1, cin, G});
      const auto& bc = need(wm, s + "residual_block_cin_conv" + ln + "bias", {G});
      for (int i = 0; i < cin; ++i)
        for (int g = 0; g < G; ++g) condw[(size_t)i * L * G + (size_t)l * G + g] = kc.data[(size_t)i * G + g];
      for (int g = 0; g < G; ++g) condb[(size_t)l * G + g] = bc.data[g];
    }
    if (c->cfg.gin_channels > 0) {
      (void)need(wm, s + "residual_block_gin_conv" + ln + "kernel", {1, c->cfg.gin_channels, G});
      (void)need(wm, s + "residual_block_gin_conv" + ln + "bias", {G});
    }
  }
  if (c->cfg.gin_channels > 0 && c->cfg.n_speakers > 0)
    (void)need(wm, "WaveNet_model/gc_embedding", {c->cfg.n_speakers, c->cfg.gin_channels});
  c->gc_B = 0;
  wupload(c->conv_w, cw);
  wupload(c->conv_b, cb);
  wupload(c->so_w, sow);
  wupload(c->so_b, sob);
  wupload(c->cond_w, condw);
  wupload(c->cond_b, condb);
  wupload(c->f1_w, need(wm, P + "skip_convolutions/final_convolution_1/kernel", {1, S, S}).data);
  wupload(c->f1_b, need(wm, P + "skip_convolutions/final_convolution_1/bias", {S}).data);
  wupload(c->f2_w, need(wm, P + "skip_convolutions/final_convolution_2/kernel", {1, S, Q}).data);
  wupload(c->f2_b, need(wm, P + "skip_convolutions/final_convolution_2/bias", {Q}).data);
  wn_upload_upsampler(c);
  c->finalized = true;
}

static void wn_finalize(tt2_wn_ctx* c) {
  if (c->quantize) {
    wn_finalize_q(c);
    return;
  }
  const WeightMap& wm = c->host;
  const std::string P(WP);
  const int R = c->R, G = c->G, S = c->S, L = c->L, C = c->C, cin = c->cin, kw = c->cfg.kernel_size;
  TT2_HIP(hipSetDevice(c->dev));
  wupload(c->first_w, need(wm, P + "input_convolution/kernel", {1, 1, R}).data);
  wupload(c->first_b, need(wm, P + "input_convolution/bias", {R}).data);
  constexpr int CK = WN_CK, SK = WN_SK;
  std::vector<float> cw((size_t)L * CK * WN_THREADS * 4), cb((size_t)L * G), condw((size_t)std::max(cin, 1) * L * G, 0.f),
      condb((size_t)L * G), sow((size_t)L * SK * WN_THREADS * 4), sob((size_t)L * 2 * R);
  std::vector<float> wide_cw, wide_so;
  if (c->wide) {
    cw.clear();
    sow.clear();
  }
  for (int l = 0; l < L; ++l) {
    const std::string s = P + "ResidualConv1DGLU_" + std::to_string(l) + "/";
    const std::string ln = "_ResidualConv1DGLU_" + std::to_string(l) + "/";
    const auto& k = need(wm, s + "residual_block_causal_conv" + ln + "kernel", {kw, R, G});
    const auto& bb = need(wm, s + "residual_block_causal_conv" + ln + "bias", {G});
    // local conditioning off (cin_channels <= 0): no conv1x1c (modules.py:416-424)
    const HostTensor* kc = cin > 0 ? &need(wm, s + "residual_block_cin_conv" + ln + "kernel", {1, cin, G}) : nullptr;
    const HostTensor* bc = cin > 0 ? &need(wm, s + "residual_block_cin_conv" + ln + "bias", {G}) : nullptr;
    const auto& ksk = need(wm, s + "residual_block_skip_conv" + ln + "kernel", {1, G / 2, S});
    const auto& bsk = need(wm, s + "residual_block_skip_conv" + ln + "bias", {S});
    const auto& ko = need(wm, s + "residual_block_out_conv" + ln + "kernel", {1, G / 2, R});
    const auto& bo = need(wm, s + "residual_block_out_conv" + ln + "bias", {R});
    if (c->wide) {  // k_generate_wide: gate-column blocks of ww_nc(R) work-groups per layer
      for (int cc = 0; cc < ww_nc(R); ++cc) {
        ww_pack_conv(k.data.data(), R, cc, wide_cw);
        ww_pack_so(ksk.data.data(), ko.data.data(), R, cc, wide_so);
      }
    }
    for (int tid = 0; tid < (c->wide ? 0 : WN_THREADS); ++tid) {
      const int q = tid / 8, ks = tid % 8;  // 32 column quads x 8 k-slices
      for (int kk = 0; kk < CK; ++kk) {
        // row of the linearized [kw*R, G] kernel (taps oldest first): kk < 16 -> tap row 16ks+kk
        // of [x(t-2d) | x(t-d)], kk >= 16 -> x(t) row 2R + 8ks + (kk-16)
        const int kidx = kk < WN_TK ? WN_TK * ks + kk : 2 * R + WN_XK * ks + (kk - WN_TK);
        for (int e = 0; e < 4; ++e)
          cw[(((size_t)l * CK + kk) * WN_THREADS + tid) * 4 + e] = k.data[(size_t)kidx * G + gate_col(R, q, e)];
      }
      for (int kk = 0; kk < SK; ++kk) {
        const int kidx = ks * SK + kk;
        for (int e = 0; e < 4; ++e) {
          const int col = 4 * q + e;  // 0..127: [skip 0..63 | out 0..63]
          const float v = col < S ? ksk.data[(size_t)kidx * S + col] : ko.data[(size_t)kidx * R + (col - S)];
          sow[(((size_t)l * SK + kk) * WN_THREADS + tid) * 4 + e] = v;
        }
      }
    }
    for (int q = 0; q < G / 4; ++q)
      for (int e = 0; e < 4; ++e) {
        const int src = gate_col(R, q, e), dst = 4 * q + e;
        cb[(size_t)l * G + dst] = bb.data[src];
        condb[(size_t)l * G + dst] = bc ? bc->data[src] : 0.f;
        for (int i = 0; i < cin; ++i) condw[(size_t)i * L * G + l * G + dst] = kc->data[(size_t)i * G + src];
      }
    for (int j = 0; j < S; ++j) sob[(size_t)l * 2 * R + j] = bsk.data[j];
    for (int j = 0; j < R; ++j) sob[(size_t)l * 2 * R + S + j] = bo.data[j];
  }
  wupload(c->conv_w, c->wide ? wide_cw : cw);
  wupload(c->conv_b, cb);
  if (c->wide && ww_onehop(R)) {  // one-hop R = 256 form: per layer M = rs·W_x(l)·O(l-1), folded biases
    TT2_CHECK(R == 256 && G == 512 && S == 256, TT2_ERR_INVALID_ARG, "one-hop wide WaveNet needs R = 256");
    const float rs = c->cfg.residual_legacy ? 0.70710677f : 1.f;
    std::vector<float> w1, gb1((size_t)L * G);
    std::vector<double> M((size_t)R * G);
    const float* prev_o = nullptr;
    const float* prev_s = nullptr;
    const float* prev_bo = nullptr;
    for (int l = 0; l <= L; ++l) {
      const float* conv = nullptr;
      const float* ko = nullptr;
      const float* ksk = nullptr;
      const float* bo = nullptr;
      if (l < L) {
        const std::string s = P + "ResidualConv1DGLU_" + std::to_string(l) + "/";
        const std::string ln = "_ResidualConv1DGLU_" + std::to_string(l) + "/";
        conv = need(wm, s + "residual_block_causal_conv" + ln + "kernel", {kw, R, G}).data.data();
        ko = need(wm, s + "residual_block_out_conv" + ln + "kernel", {1, G / 2, R}).data.data();
        ksk = need(wm, s + "residual_block_skip_conv" + ln + "kernel", {1, G / 2, S}).data.data();
        bo = need(wm, s + "residual_block_out_conv" + ln + "bias", {R}).data.data();
        for (int q = 0; q < G / 4; ++q)  // gate bias + rs·W_x(l)·bo(l-1), gate-permuted like conv_b
          for (int e = 0; e < 4; ++e) {
            const int src = gate_col(R, q, e);
            double v = cb[(size_t)l * G + 4 * q + e];
            if (prev_bo) {
              double acc = 0.0;
              for (int x = 0; x < R; ++x) acc += (double)conv[(size_t)(2 * R + x) * G + src] * prev_bo[x];
              v += rs * acc;
            }
            gb1[(size_t)l * G + 4 * q + e] = (float)v;
          }
        if (prev_o) {  // M[z][g] = rs · Σ_x O(l-1)[z][x] · W_x(l)[x][g]
          for (int z = 0; z < R; ++z) {
            double* mr = M.data() + (size_t)z * G;
            for (int g = 0; g < G; ++g) mr[g] = 0.0;
            for (int x = 0; x < R; ++x) {
              const double o = prev_o[(size_t)z * R + x];
              const float* wr = conv + (size_t)(2 * R + x) * G;
              for (int g = 0; g < G; ++g) mr[g] += o * wr[g];
            }
            for (int g = 0; g < G; ++g) mr[g] *= rs;
          }
        }
      }
      for (int cc = 0; cc < ww_nc(R); ++cc) ww1_pack(conv, prev_o, prev_s, prev_o && conv ? M.data() : nullptr, rs, cc, w1);
      prev_o = ko;
      prev_s = ksk;
      prev_bo = bo;
    }
    wupload(c->w1, w1);
    wupload(c->gb1, gb1);
    {  // layer 0 folded into the head (WideArgs::l0): U_k = W_k·fw, V_k = W_k·fb per gate column
      const std::string s = P + "ResidualConv1DGLU_0/";
      const float* conv = need(wm, s + "residual_block_causal_conv_ResidualConv1DGLU_0/kernel", {kw, R, G}).data.data();
      const float* fw = need(wm, P + "input_convolution/kernel", {1, 1, R}).data.data();
      const float* fb = need(wm, P + "input_convolution/bias", {R}).data.data();
      std::vector<float> l0((size_t)R * 16, 0.f);
      for (int j = 0; j < R; ++j)
        for (int h = 0; h < 2; ++h) {
          const int col = h ? R + j : j;
          float* o = l0.data() + (size_t)j * 16 + h * 8;
          for (int k = 0; k < 3; ++k) {
            double u = 0.0, v = 0.0;
            for (int x = 0; x < R; ++x) {
              const double w = conv[(size_t)(k * R + x) * G + col];
              u += w * fw[x];
              v += w * fb[x];
            }
            o[k] = (float)u;
            o[4 + k] = (float)v;
          }
          o[3] = gb1[4 * (j >> 1) + (j & 1) + 2 * h];  // gate bias, gate-permuted column
        }
      wupload(c->l0, l0);
    }
  }
  if (c->cfg.gin_channels > 0) {  // conv1x1g of every layer (modules.py:427-433) and the embedding
    for (int l = 0; l < L; ++l) {
      const std::string s = P + "ResidualConv1DGLU_" + std::to_string(l) + "/";
      const std::string ln = "_ResidualConv1DGLU_" + std::to_string(l) + "/";
      (void)need(wm, s + "residual_block_gin_conv" + ln + "kernel", {1, c->cfg.gin_channels, G});
      (void)need(wm, s + "residual_block_gin_conv" + ln + "bias", {G});
    }
    if (c->cfg.n_speakers > 0) (void)need(wm, "WaveNet_model/gc_embedding", {c->cfg.n_speakers, c->cfg.gin_channels});
  }
  c->gc_B = 0;
  wupload(c->cond_w, condw);
  wupload(c->cond_b, condb);
  wupload(c->so_w, c->wide ? wide_so : sow);
  wupload(c->so_b, sob);
  wupload(c->f1_w, need(wm, P + "skip_convolutions/final_convolution_1/kernel", {1, S, S}).data);
  wupload(c->f1_b, need(wm, P + "skip_convolutions/final_convolution_1/bias", {S}).data);
  wupload(c->f2_w, need(wm, P + "skip_convolutions/final_convolution_2/kernel", {1, S, C}).data);
  wupload(c->f2_b, need(wm, P + "skip_convolutions/final_convolution_2/bias", {C}).data);
  wn_upload_upsampler(c);
  c->finalized = true;
}

typedef void (*PipeKernel)(GenArgs);
static PipeKernel pipe_kernel(bool legacy, bool res_legacy, bool gauss) {
  if (gauss) {
    if (legacy) return res_legacy ? k_generate_pipe<true, true, true> : k_generate_pipe<true, false, true>;
    return res_legacy ? k_generate_pipe<false, true, true> : k_generate_pipe<false, false, true>;
  }
  if (legacy) return res_legacy ? k_generate_pipe<true, true, false> : k_generate_pipe<true, false, false>;
  return res_legacy ? k_generate_pipe<false, true, false> : k_generate_pipe<false, false, false>;
}

// the generation kernel's bounded spins report a stalled hand-off through the status word
static void check_status(tt2_wn_ctx* c) {
  TT2_CHECK(*c->status_host == 0, TT2_ERR_HIP,
            "WaveNet generation: a pipeline hand-off timed out (stage workgroups not co-resident?)");
}

static int wn_stages(const tt2_wn_ctx* c) { return (c->L + WN_LPS - 1) / WN_LPS; }

static size_t gen_lds_bytes(const tt2_wn_ctx* c) {
  const int per = c->L / c->cfg.stacks, nst = wn_stages(c);
  long ring = 0;
  for (int st = 0; st < nst; ++st) {
    long r = 0;
    for (int l = st * WN_LPS; l < std::min(c->L, (st + 1) * WN_LPS); ++l) r += (2 * (1 << (l % per)) + 1) * c->R;
    ring = std::max(ring, r);
  }
  const long fixed = 64 + 64 * 6 + 32 + 32 + 2 * WN_LPS * 128 + 2 * WN_LPS * 128 + 64 * 64 + 64 * 32 + 100;
  return sizeof(float) * (fixed + ring);
}

// Read-back of the device RNG streams of k_generate_pipe (tt2_wn_noise): row r = t*Bg + b.
__global__ void k_wn_noise(uint64_t seed, long n, int Bg, int nr, int gaussian, float* __restrict__ um,
                           float* __restrict__ ul) {
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < n; r += (long)gridDim.x * blockDim.x) {
    const long t = r / Bg;
    const int b = (int)(r % Bg);
    if (gaussian) {
      ul[r] = wn_gauss(seed, t, Bg, b);
    } else {
      for (int c = 0; c < nr; ++c) um[r * nr + c] = wn_uniform(seed, t, Bg, b, c);
      ul[r] = wn_uniform(seed, t, Bg, b, 15);
    }
  }
}

static void wn_generate_dev(tt2_wn_ctx* c, const float* cond_in, int B, int T_f, const float* umix_d,
                            const float* ulog_d, uint64_t seed, const float* teacher_d, float* wav_d, int* k_d,
                            float* logits_d, float* upsampled_d, hipStream_t s, long T_uncond = 0) {
  TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_wn_finalize not called");
  TT2_CHECK(B >= 1 && B <= c->cfg.max_batch, TT2_ERR_SHAPE_MISMATCH, "batch exceeds capacity");
  // cond_in null: unconditional synthesis of T_uncond samples (wavenet.py:410-411)
  const bool uncond = cond_in == nullptr;
  TT2_CHECK(uncond == (c->cin == 0), TT2_ERR_INVALID_ARG,
            uncond ? "local conditioning on (cin_channels > 0): a condition is required"
                   : "cin_channels <= 0: unconditional synthesis (tt2_wn_generate_unconditional)");
  const long T = uncond ? T_uncond : (long)T_f * c->hop;
  TT2_CHECK((uncond || T_f >= 1) && T >= 1 && T <= c->cfg.max_samples, TT2_ERR_SHAPE_MISMATCH,
            "synthesis length exceeds capacity");
  const int F = c->cin;
  TT2_HIP(hipEventRecord(c->ev[0], s));
  const bool need_cond = !uncond || c->cfg.gin_channels > 0 || !c->quantize;
  if (uncond) {  // no conv1x1c term: zero conditioning (+ the global term below)
    TT2_HIP(hipEventRecord(c->ev[1], s));
    if (need_cond) {
      c->cond.alloc(sizeof(float) * B * T * c->L * c->G);
      TT2_HIP(hipMemsetAsync(c->cond.p, 0, sizeof(float) * B * T * c->L * c->G, s));
    }
  } else {
  // upsampling network: [B][F][T_f] -> [B][F][T]
  c->up_a.alloc(sizeof(float) * B * F * T);
  c->up_b_buf.alloc(sizeof(float) * B * F * T);
  c->c_up_t.alloc(sizeof(float) * B * T * F);
  const float* src = cond_in;  // [B][F][T_f] channels-first
  long Tcur = T_f;
  float* bufs[2] = {c->up_a.as<float>(), c->up_b_buf.as<float>()};
  const int ut = c->cfg.upsample_type;
  const int nup = ut == WN_UP_NN ? 1 : c->cfg.n_upsample;  // NearestNeighborUpsample: one x hop layer
  const int act = ut == WN_UP_NN ? WN_ACT_NONE : c->cfg.upsample_activation;
  for (int i = 0; i < nup; ++i) {
    const int sc = ut == WN_UP_NN ? (int)c->hop : c->cfg.upsample_scales[i];
    const bool last = i + 1 == nup;
    float* dst = (last && upsampled_d) ? upsampled_d : bufs[i & 1];
    const long n = (long)B * F * Tcur * sc;
    const int grid = (int)std::min<long>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(k_upsample, dim3(grid), dim3(256), 0, s, src, dst, last ? c->c_up_t.as<float>() : nullptr,
                       ut == WN_UP_NN ? nullptr : c->up_k[i].as<float>(), ut == WN_UP_NN ? nullptr : c->up_b[i].as<float>(),
                       B, F, (int)Tcur, sc, c->cfg.freq_axis_kernel_size, ut, act, c->cfg.leaky_alpha);
    TT2_HIP(hipGetLastError());
    src = dst;
    Tcur *= sc;
  }
  TT2_HIP(hipEventRecord(c->ev[1], s));
  // conditioning 1x1 of every layer for every sample: [B*T, F] x [F, L*G]
  c->cond.alloc(sizeof(float) * B * T * c->L * c->G);
  GemmArgs g;
  g.M = (int)(B * T); g.N = c->L * c->G; g.K = F; g.A = c->c_up_t.as<float>(); g.lda = F;
  g.Bw = c->cond_w.as<float>(); g.ldb = c->L * c->G; g.Cout = c->cond.as<float>(); g.ldc = c->L * c->G;
  g.bias = c->cond_b.as<float>();
  g.split16 = 1;  // conditioning in [0, 1] after the upsampler: fp16x3 split MFMA (gemm.h)
  gemm(g, s);
  }
  if (c->cfg.gin_channels > 0) {  // + g·W_g + b_g of every layer (constant over time)
    TT2_CHECK(c->gc_B == B, TT2_ERR_STATE,
              "gin_channels > 0: tt2_wn_set_global_condition for exactly these B rows before generating");
    const long n = (long)B * T * c->L * c->G;
    hipLaunchKernelGGL(k_add_gc, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c->cond.as<float>(),
                       c->gcv.as<float>(), B, (long)T, c->L * c->G);
    TT2_HIP(hipGetLastError());
  }
  TT2_HIP(hipEventRecord(c->ev[2], s));
  if (c->quantize) {  // one-hot input, Q-class softmax head (wavenet_q.hip)
    const int per = c->L / c->cfg.stacks;
    const long rf = wq_ring_floats(c->R, c->L, per);
    c->rings.alloc(sizeof(float) * B * rf);
    TT2_HIP(hipMemsetAsync(c->rings.p, 0, sizeof(float) * B * rf, s));
    QGenArgs q{};
    q.T = (int)T; q.L = c->L; q.per = per; q.R = c->R; q.G = c->G; q.S = c->S; q.Q = c->C; q.Bg = B;
    q.legacy = c->cfg.legacy; q.res_legacy = c->cfg.residual_legacy;
    q.k0 = 127;  // mulaw_quantize(0) = int((0 + 1) / 2 * 255), mu hard-coded to 255 (util.py:71-102)
    q.first_w = c->first_w.as<float>(); q.first_b = c->first_b.as<float>();
    q.conv_w = c->conv_w.as<float>(); q.conv_b = c->conv_b.as<float>();
    q.cond = need_cond ? c->cond.as<float>() : nullptr;
    q.so_w = c->so_w.as<float>(); q.so_b = c->so_b.as<float>();
    q.f1_w = c->f1_w.as<float>(); q.f1_b = c->f1_b.as<float>(); q.f2_w = c->f2_w.as<float>(); q.f2_b = c->f2_b.as<float>();
    q.u = ulog_d; q.seed = seed; q.teacher = teacher_d;
    q.wav = wav_d; q.kout = k_d; q.logits = logits_d;
    q.rings = c->rings.as<float>(); q.ring_floats = rf;
    wq_launch(q, s);
    *c->status_host = 0;
    TT2_HIP(hipEventRecord(c->ev[3], s));
    c->timed = true;
    return;
  }
  if (c->wide) {
    const int R = c->R, NG = ww_nc(R) * 2 * R;
    c->rings.alloc(sizeof(float) * ww_ring_floats(R, c->L, c->L / c->cfg.stacks));
    const size_t gbytes = sizeof(unsigned long long) * ((size_t)c->L * NG + 1) + 16;
    c->gran.alloc(gbytes);
    WideArgs w;
    w.T = (int)T; w.L = c->L; w.per = c->L / c->cfg.stacks; w.Bg = B;
    w.first_w = c->first_w.as<float>(); w.first_b = c->first_b.as<float>();
    w.conv_w = c->conv_w.as<f32x4>(); w.conv_b = c->conv_b.as<float>(); w.cond = c->cond.as<float>();
    w.so_w = c->so_w.as<f32x4>(); w.so_b = c->so_b.as<float>();
    w.f1_w = c->f1_w.as<float>(); w.f1_b = c->f1_b.as<float>(); w.f2_w = c->f2_w.as<float>(); w.f2_b = c->f2_b.as<float>();
    w.C = c->C; w.legacy = c->cfg.legacy; w.res_legacy = c->cfg.residual_legacy;
    w.log_scale_min = c->cfg.log_scale_min; w.log_scale_min_gauss = c->cfg.log_scale_min_gauss;
    w.u_mix = umix_d; w.u_log = ulog_d; w.seed = seed; w.teacher = teacher_d;
    w.wav = wav_d; w.kout = k_d; w.logits = logits_d;
    w.rings = c->rings.as<float>();
    w.status = c->gran.as<int>();
    w.gran = reinterpret_cast<unsigned long long*>(c->gran.as<char>() + 16);
    w.w1 = c->w1.p ? c->w1.as<f32x4>() : nullptr;
    w.gb1 = c->gb1.p ? c->gb1.as<float>() : nullptr;
    static const bool fuse0 = [] {
      const char* e = std::getenv("TT2_WW_L0HEAD");  // 0: layer 0 on its own work-groups (A/B)
      return !e || std::atoi(e) != 0;
    }();
    w.l0 = fuse0 && c->l0.p ? c->l0.as<float>() : nullptr;
    const void* kern = ww_kernel(R, c->C == 2);
    const unsigned shm = (unsigned)ww_lds_bytes(R, c->C);
    for (int b = 0; b < B; ++b) {  // one utterance per launch: its layers fill NC x L CUs
      w.b = b;
      TT2_HIP(hipMemsetAsync(c->gran.p, 0, gbytes, s));  // every polled word starts at 0
      void* params[] = {&w};
      TT2_HIP(launch_persistent(kern, dim3(ww_blocks(R, c->L)), dim3(WW_THREADS), params, shm, s));
      TT2_HIP(hipMemcpyAsync(c->status_host, c->gran.p, sizeof(int), hipMemcpyDeviceToHost, s));
    }
    TT2_HIP(hipEventRecord(c->ev[3], s));
    c->timed = true;
    return;
  }
  const int nst = wn_stages(c);
  const int chunk = c->chunk;  // utterances per launch: every stage of every utterance co-resident
  const size_t gbytes = sizeof(unsigned long long) * (size_t)chunk * nst * WN_GR + 16;
  c->gran.alloc(gbytes);
  GenArgs a;
  a.T = (int)T; a.L = c->L; a.per = c->L / c->cfg.stacks; a.nst = nst; a.Bg = B;
  a.first_w = c->first_w.as<float>(); a.first_b = c->first_b.as<float>();
  a.conv_w = c->conv_w.as<f32x4>(); a.conv_b = c->conv_b.as<float>(); a.cond = c->cond.as<float>();
  a.so_w = c->so_w.as<f32x4>(); a.so_b = c->so_b.as<float>();
  a.f1_w = c->f1_w.as<float>(); a.f1_b = c->f1_b.as<float>(); a.f2_w = c->f2_w.as<float>(); a.f2_b = c->f2_b.as<float>();
  a.C = c->C; a.legacy = c->cfg.legacy; a.res_legacy = c->cfg.residual_legacy; a.log_scale_min = c->cfg.log_scale_min;
  a.log_scale_min_gauss = c->cfg.log_scale_min_gauss;
  a.u_mix = umix_d; a.u_log = ulog_d; a.seed = seed; a.teacher = teacher_d;
  a.wav = wav_d; a.kout = k_d; a.logits = logits_d;
  a.status = c->gran.as<int>();
  c->stamps.alloc(sizeof(long long) * 64 * 8);
  TT2_HIP(hipMemsetAsync(c->stamps.p, 0, sizeof(long long) * 64 * 8, s));
  a.stamps = c->stamps.as<long long>();
  a.gran = reinterpret_cast<unsigned long long*>(c->gran.as<char>() + 16);
  const size_t shm = gen_lds_bytes(c);
  for (int b0 = 0; b0 < B; b0 += chunk) {
    a.b0 = b0;
    a.B = std::min(chunk, B - b0);
    // every polled word (granule tags, status) starts at 0 for each launch (Guideline 16)
    TT2_HIP(hipMemsetAsync(c->gran.p, 0, gbytes, s));
    const int grid = cdiv(a.B, 8) * nst * 8;
    const auto kern = pipe_kernel(c->cfg.legacy != 0, c->cfg.residual_legacy != 0, c->C == 2);
    // cooperative: every stage work-group of the launch co-resident (the stage hand-offs spin)
    void* params[] = {&a};
    TT2_HIP(launch_persistent(reinterpret_cast<const void*>(kern), dim3(grid), dim3(WN_THREADS), params,
                                       (unsigned)shm, s));
    TT2_HIP(hipMemcpyAsync(c->status_host, c->gran.p, sizeof(int), hipMemcpyDeviceToHost, s));
  }
  TT2_HIP(hipEventRecord(c->ev[3], s));
  c->timed = true;
}

}  // namespace tt2

using namespace tt2;

extern "C" {

void tt2_wn_default_config(tt2_wn_config* c, int max_batch, int64_t max_samples) {
  std::memset(c, 0, sizeof(*c));
  c->layers = 24; c->stacks = 4; c->residual_channels = 64; c->gate_channels = 128; c->skip_out_channels = 64;
  c->kernel_size = 3; c->cin_channels = 80; c->out_channels = 30; c->legacy = 0; c->residual_legacy = 0;
  c->log_scale_min = (float)std::log(1e-14); c->n_upsample = 3;
  c->upsample_scales[0] = 5; c->upsample_scales[1] = 5; c->upsample_scales[2] = 11;
  c->freq_axis_kernel_size = 3; c->max_batch = max_batch; c->max_samples = max_samples;
  c->upsample_type = 0; c->upsample_activation = 1; c->leaky_alpha = 0.4f; c->NN_init = 1;
  c->log_scale_min_gauss = (float)std::log(1e-7);
  c->gin_channels = -1; c->n_speakers = 0;
  c->input_type = 0; c->quantize_channels = 256;
}

tt2_status tt2_wn_create(const tt2_wn_config* cfg, int hip_device, tt2_wn_ctx** out) {
  return guard([&] {
    TT2_CHECK(cfg && out, TT2_ERR_INVALID_ARG, "tt2_wn_create: null argument");
    *out = nullptr;
    int ndev = 0;
    TT2_HIP(hipGetDeviceCount(&ndev));
    TT2_CHECK(hip_device >= 0 && hip_device < ndev, TT2_ERR_INVALID_ARG, "tt2_wn_create: bad device index");
    const int Rc = cfg->residual_channels;
    TT2_CHECK((Rc == 64 || Rc == 128 || Rc == 256) && cfg->gate_channels == 2 * Rc && cfg->skip_out_channels == Rc,
              TT2_ERR_INVALID_ARG,
              "generation kernels: residual_channels R = 64 (k_generate_pipe, BASELINE config 3), 128 (fork "
              "default) or 256 (paper default), with gate_channels = 2R and skip_out_channels = R");
    TT2_CHECK(cfg->kernel_size == 3, TT2_ERR_INVALID_ARG, "kernel_size must be 3");
    TT2_CHECK(cfg->input_type >= 0 && cfg->input_type <= 2, TT2_ERR_INVALID_ARG,
              "input_type: 0 'raw', 1 'mulaw', 2 'mulaw-quantize'");
    const bool quant = cfg->input_type == 2;
    if (quant)
      TT2_CHECK(cfg->out_channels == cfg->quantize_channels && cfg->quantize_channels >= 4 &&
                    cfg->quantize_channels <= WQ_QMAX && cfg->quantize_channels % 4 == 0,
                TT2_ERR_INVALID_ARG,
                "mulaw-quantize: out_channels must equal quantize_channels (a multiple of 4, <= 1024)");
    else
      TT2_CHECK(cfg->out_channels == 2 || (cfg->out_channels % 3 == 0 && cfg->out_channels <= 30 && cfg->out_channels >= 3),
                TT2_ERR_INVALID_ARG, "head needs out_channels = 2 (Gaussian) or 3*nr_mix <= 30 (MoL)");
    TT2_CHECK(cfg->layers >= 1 && cfg->stacks >= 1 && cfg->layers % cfg->stacks == 0, TT2_ERR_INVALID_ARG,
              "layers % stacks != 0");
    TT2_CHECK(cfg->cin_channels <= 128, TT2_ERR_INVALID_ARG, "cin_channels out of range");
    if (cfg->cin_channels > 0) {  // local conditioning: the upsampling network
      TT2_CHECK(cfg->upsample_type >= WN_UP_2D && cfg->upsample_type <= WN_UP_NN, TT2_ERR_INVALID_ARG,
                "upsample_type out of range");
      TT2_CHECK(cfg->upsample_activation >= WN_ACT_NONE && cfg->upsample_activation <= WN_ACT_LEAKY,
                TT2_ERR_INVALID_ARG, "upsample_activation out of range");
      TT2_CHECK(cfg->n_upsample >= 1 && cfg->n_upsample <= 8, TT2_ERR_INVALID_ARG, "n_upsample out of range");
    }
    TT2_CHECK(cfg->max_batch >= 1 && cfg->max_samples >= 1, TT2_ERR_INVALID_ARG, "capacities must be >= 1");
    auto c = std::make_unique<tt2_wn_ctx>();
    c->cfg = *cfg;
    c->dev = hip_device;
    c->R = cfg->residual_channels; c->G = cfg->gate_channels; c->S = cfg->skip_out_channels;
    c->L = cfg->layers; c->C = cfg->out_channels; c->cin = std::max(cfg->cin_channels, 0);
    c->hop = 1;
    for (int i = 0; c->cin > 0 && i < cfg->n_upsample; ++i) c->hop *= cfg->upsample_scales[i];
    TT2_HIP(hipSetDevice(hip_device));
    TT2_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (auto& e : c->ev) TT2_HIP(hipEventCreate(&e));
    if (quant) {  // k_generate_q: one work-group per utterance, no co-residency requirement
      c->quantize = true;
      const size_t qshm = wq_lds_bytes(c->R, c->G, c->S, c->C);
      TT2_CHECK(qshm <= 64 * 1024, TT2_ERR_INVALID_ARG, "mulaw-quantize generator LDS exceeds 64 KiB");
      TT2_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->status_host), sizeof(int), hipHostMallocDefault));
      *c->status_host = 0;
      *out = c.release();
      return;
    }
    int ncu = 0;
    TT2_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, hip_device));
    if (Rc != 64) {  // k_generate_wide: NC work-groups per layer + a head, queues in global memory
      c->wide = true;
      const void* wk = ww_kernel(Rc, cfg->out_channels == 2);
      const size_t wshm = ww_lds_bytes(Rc, cfg->out_channels);
      TT2_HIP(hipFuncSetAttribute(wk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wshm));
      int nbw = 0;
      TT2_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nbw, wk, WW_THREADS, wshm));
      TT2_CHECK(nbw >= 1, TT2_ERR_INVALID_ARG, "wide generation kernel does not fit on a CU");
      TT2_CHECK(ww_blocks(Rc, cfg->layers) <= ncu, TT2_ERR_INVALID_ARG,
                "wide WaveNet: layers x work-groups per layer + head exceed the device's CUs");
      c->chunk = 1;
      TT2_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->status_host), sizeof(int), hipHostMallocDefault));
      *c->status_host = 0;
      *out = c.release();
      return;
    }
    const size_t shm = gen_lds_bytes(c.get());
    TT2_CHECK(shm <= 160 * 1024, TT2_ERR_INVALID_ARG, "queue rings exceed the 160 KiB LDS of a CU");
    const void* kern = reinterpret_cast<const void*>(pipe_kernel(cfg->legacy != 0, cfg->residual_legacy != 0, cfg->out_channels == 2));
    TT2_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    // co-residency: one stage workgroup per CU, every workgroup of a launch resident at once
    int nb = 0;
    TT2_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, WN_THREADS, shm));
    TT2_CHECK(nb >= 1, TT2_ERR_INVALID_ARG, "generation kernel does not fit on a CU");
    const int nst = wn_stages(c.get());
    TT2_CHECK(nst * 8 <= ncu, TT2_ERR_INVALID_ARG, "too many pipeline stages for this device");
    c->chunk = 8 * (ncu / (nst * 8));  // grid = ceil(chunk/8)*nst*8 <= ncu
    TT2_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->status_host), sizeof(int), hipHostMallocDefault));
    *c->status_host = 0;
    *out = c.release();
  });
}

tt2_status tt2_wn_set_global_condition(tt2_wn_ctx* c, const int32_t* ids, const float* feat, int B) {
  return guard([&] {
    TT2_CHECK(c && c->finalized, TT2_ERR_NOT_LOADED, "tt2_wn_set_global_condition: not finalized");
    const int gin = c->cfg.gin_channels, L = c->L, G = c->G, R = c->R;
    TT2_CHECK(gin > 0, TT2_ERR_STATE, "global conditioning off (gin_channels <= 0)");
    if (!ids && !feat) {
      c->gc_B = 0;
      return;
    }
    TT2_CHECK(B >= 1 && B <= c->cfg.max_batch, TT2_ERR_SHAPE_MISMATCH, "B out of [1, max_batch]");
    TT2_CHECK(!ids || c->cfg.n_speakers > 0, TT2_ERR_INVALID_ARG,
              "speaker ids need the gc_embedding table (n_speakers > 0, use_speaker_embedding)");
    const WeightMap& wm = c->host;
    std::vector<float> g((size_t)B * gin);
    for (int b = 0; b < B; ++b) {
      if (ids) {  // embedding_lookup (modules.py:13-23)
        const auto& emb = need(wm, "WaveNet_model/gc_embedding", {c->cfg.n_speakers, gin});
        TT2_CHECK(ids[b] >= 0 && ids[b] < c->cfg.n_speakers, TT2_ERR_INVALID_ARG, "speaker id out of range");
        std::copy(emb.data.begin() + (size_t)ids[b] * gin, emb.data.begin() + (size_t)(ids[b] + 1) * gin,
                  g.begin() + (size_t)b * gin);
      } else {
        std::copy(feat + (size_t)b * gin, feat + (size_t)(b + 1) * gin, g.begin() + (size_t)b * gin);
      }
    }
    std::vector<float> gcv((size_t)B * L * G);
    const std::string P(WP);
    for (int l = 0; l < L; ++l) {
      const std::string s = P + "ResidualConv1DGLU_" + std::to_string(l) + "/";
      const std::string ln = "_ResidualConv1DGLU_" + std::to_string(l) + "/";
      const auto& kg = need(wm, s + "residual_block_gin_conv" + ln + "kernel", {1, gin, G});
      const auto& bg = need(wm, s + "residual_block_gin_conv" + ln + "bias", {G});
      for (int b = 0; b < B; ++b)
        for (int q = 0; q < G / 4; ++q)
          for (int e = 0; e < 4; ++e) {
            // the conditioning's gate permutation (natural order for k_generate_q)
            const int src = c->quantize ? 4 * q + e : gate_col(R, q, e), dst = 4 * q + e;
            double v = bg.data[src];
            for (int i = 0; i < gin; ++i) v += (double)g[(size_t)b * gin + i] * kg.data[(size_t)i * G + src];
            gcv[((size_t)b * L + l) * G + dst] = (float)v;
          }
    }
    TT2_HIP(hipSetDevice(c->dev));
    wupload(c->gcv, gcv);
    c->gc_B = B;
  });
}

void tt2_wn_destroy(tt2_wn_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->status_host) (void)hipHostFree(c->status_host);
  delete c;
}

tt2_status tt2_wn_last_timings(tt2_wn_ctx* c, float* ms3) {
  return guard([&] {
    TT2_CHECK(c && ms3, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->timed, TT2_ERR_STATE, "no generate call yet");
    TT2_HIP(hipEventSynchronize(c->ev[3]));
    TT2_HIP(hipStreamSynchronize(c->stream));
    check_status(c);
    for (int i = 0; i < 3; ++i) TT2_HIP(hipEventElapsedTime(&ms3[i], c->ev[i], c->ev[i + 1]));
  });
}

tt2_status tt2_wn_debug_stamps(tt2_wn_ctx* c, long long* out512) {
  return guard([&] {
    TT2_CHECK(c && out512, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->stamps.p, TT2_ERR_STATE, "no generate call yet");
    TT2_HIP(hipStreamSynchronize(c->stream));
    TT2_HIP(hipMemcpy(out512, c->stamps.p, sizeof(long long) * 512, hipMemcpyDeviceToHost));
  });
}

tt2_status tt2_wn_load_tensor(tt2_wn_ctx* c, const char* name, const float* host, const int64_t* shape, int ndim) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    put_tensor(c->host, name, host, shape, ndim);
    c->finalized = false;
  });
}

tt2_status tt2_wn_finalize(tt2_wn_ctx* c) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    wn_finalize(c);
  });
}

// 'mulaw-quantize' teacher inputs are class indices: integers in [0, quantize_channels) (host check
// of the tt2_wn_generate* host-buffer entry points; the device-pointer variant clamps in the kernel)
static void wn_check_teacher(const tt2_wn_ctx* c, const float* teacher, long n) {
  if (!c->quantize || !teacher) return;
  for (long i = 0; i < n; ++i) {
    const float v = teacher[i];
    TT2_CHECK(v >= 0.f && v < (float)c->C && v == std::floor(v), TT2_ERR_INVALID_ARG,
              "mulaw-quantize teacher inputs must be integer classes in [0, quantize_channels)");
  }
}

tt2_status tt2_wn_generate(tt2_wn_ctx* c, const float* cond, int B, int T_f, const float* u_mix, const float* u_log,
                           uint64_t seed, const float* teacher, float* wav_out, int32_t* mix_idx_out,
                           float* logits_out, float* upsampled_out) {
  return guard([&] {
    TT2_CHECK(c && cond && wav_out, TT2_ERR_INVALID_ARG, "tt2_wn_generate: null argument");
    TT2_CHECK(B >= 1 && B <= c->cfg.max_batch && T_f >= 1, TT2_ERR_SHAPE_MISMATCH, "bad batch / length");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    const long T = (long)T_f * c->hop;
    TT2_CHECK(T <= c->cfg.max_samples, TT2_ERR_SHAPE_MISMATCH, "synthesis length exceeds capacity");
    const int F = c->cin, nr = c->quantize ? 0 : c->C / 3;
    TT2_CHECK(F > 0, TT2_ERR_INVALID_ARG, "cin_channels <= 0: tt2_wn_generate_unconditional");
    // host layout [B][T_f][F] -> device channels-first [B][F][T_f]
    std::vector<float> cf((size_t)B * F * T_f);
    for (int b = 0; b < B; ++b)
      for (int t = 0; t < T_f; ++t)
        for (int f = 0; f < F; ++f) cf[((size_t)b * F + f) * T_f + t] = cond[((size_t)b * T_f + t) * F + f];
    c->cin_d.alloc(cf.size() * sizeof(float));
    TT2_HIP(hipMemcpyAsync(c->cin_d.p, cf.data(), cf.size() * sizeof(float), hipMemcpyHostToDevice, s));
    const float *um = nullptr, *ul = nullptr, *tg = nullptr;
    if (u_mix && nr > 0) {
      c->umix.alloc(sizeof(float) * T * B * nr);
      TT2_HIP(hipMemcpyAsync(c->umix.p, u_mix, sizeof(float) * T * B * nr, hipMemcpyHostToDevice, s));
      um = c->umix.as<float>();
    }
    if (u_log) {
      c->ulog.alloc(sizeof(float) * T * B);
      TT2_HIP(hipMemcpyAsync(c->ulog.p, u_log, sizeof(float) * T * B, hipMemcpyHostToDevice, s));
      ul = c->ulog.as<float>();
    }
    wn_check_teacher(c, teacher, (long)T * B);
    if (teacher) {
      c->teacher.alloc(sizeof(float) * T * B);
      TT2_HIP(hipMemcpyAsync(c->teacher.p, teacher, sizeof(float) * T * B, hipMemcpyHostToDevice, s));
      tg = c->teacher.as<float>();
    }
    c->wav.alloc(sizeof(float) * B * T);
    c->kout.alloc(sizeof(int) * B * T);
    if (logits_out) c->logits.alloc(sizeof(float) * B * T * c->C);
    DevBuf upl;
    if (upsampled_out) upl.alloc(sizeof(float) * B * F * T);
    wn_generate_dev(c, c->cin_d.as<float>(), B, T_f, um, ul, seed, tg, c->wav.as<float>(), c->kout.as<int>(),
                    logits_out ? c->logits.as<float>() : nullptr, upsampled_out ? upl.as<float>() : nullptr, s);
    TT2_HIP(hipMemcpyAsync(wav_out, c->wav.p, sizeof(float) * B * T, hipMemcpyDeviceToHost, s));
    if (mix_idx_out) TT2_HIP(hipMemcpyAsync(mix_idx_out, c->kout.p, sizeof(int) * B * T, hipMemcpyDeviceToHost, s));
    if (logits_out)
      TT2_HIP(hipMemcpyAsync(logits_out, c->logits.p, sizeof(float) * B * T * c->C, hipMemcpyDeviceToHost, s));
    if (upsampled_out)
      TT2_HIP(hipMemcpyAsync(upsampled_out, upl.p, sizeof(float) * B * F * T, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
    check_status(c);
  });
}

tt2_status tt2_wn_generate_unconditional(tt2_wn_ctx* c, int B, int64_t T, const float* u_mix, const float* u_log,
                                         uint64_t seed, const float* teacher, float* wav_out, int32_t* mix_idx_out,
                                         float* logits_out) {
  return guard([&] {
    TT2_CHECK(c && wav_out, TT2_ERR_INVALID_ARG, "tt2_wn_generate_unconditional: null argument");
    TT2_CHECK(c->cin == 0, TT2_ERR_INVALID_ARG, "tt2_wn_generate_unconditional: cin_channels > 0 needs a condition");
    TT2_CHECK(B >= 1 && B <= c->cfg.max_batch && T >= 1 && T <= c->cfg.max_samples, TT2_ERR_SHAPE_MISMATCH,
              "bad batch / length");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    const int nr = c->quantize ? 0 : c->C / 3;
    const float *um = nullptr, *ul = nullptr, *tg = nullptr;
    if (u_mix && nr > 0) {
      c->umix.alloc(sizeof(float) * T * B * nr);
      TT2_HIP(hipMemcpyAsync(c->umix.p, u_mix, sizeof(float) * T * B * nr, hipMemcpyHostToDevice, s));
      um = c->umix.as<float>();
    }
    if (u_log) {
      c->ulog.alloc(sizeof(float) * T * B);
      TT2_HIP(hipMemcpyAsync(c->ulog.p, u_log, sizeof(float) * T * B, hipMemcpyHostToDevice, s));
      ul = c->ulog.as<float>();
    }
    wn_check_teacher(c, teacher, (long)T * B);
    if (teacher) {
      c->teacher.alloc(sizeof(float) * T * B);
      TT2_HIP(hipMemcpyAsync(c->teacher.p, teacher, sizeof(float) * T * B, hipMemcpyHostToDevice, s));
      tg = c->teacher.as<float>();
    }
    c->wav.alloc(sizeof(float) * B * T);
    c->kout.alloc(sizeof(int) * B * T);
    if (logits_out) c->logits.alloc(sizeof(float) * B * T * c->C);
    wn_generate_dev(c, nullptr, B, 0, um, ul, seed, tg, c->wav.as<float>(), c->kout.as<int>(),
                    logits_out ? c->logits.as<float>() : nullptr, nullptr, s, (long)T);
    TT2_HIP(hipMemcpyAsync(wav_out, c->wav.p, sizeof(float) * B * T, hipMemcpyDeviceToHost, s));
    if (mix_idx_out) TT2_HIP(hipMemcpyAsync(mix_idx_out, c->kout.p, sizeof(int) * B * T, hipMemcpyDeviceToHost, s));
    if (logits_out)
      TT2_HIP(hipMemcpyAsync(logits_out, c->logits.p, sizeof(float) * B * T * c->C, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
    check_status(c);
  });
}

tt2_status tt2_wn_generate_dev(tt2_wn_ctx* c, const float* cond_d, int B, int T_f, const float* u_mix_d,
                               const float* u_log_d, uint64_t seed, const float* teacher_d, float* wav_d,
                               int32_t* mix_idx_d, float* logits_d, void* stream) {
  return guard([&] {
    TT2_CHECK(c && cond_d && wav_d, TT2_ERR_INVALID_ARG, "tt2_wn_generate_dev: null argument");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    wn_generate_dev(c, cond_d, B, T_f, u_mix_d, u_log_d, seed, teacher_d, wav_d, mix_idx_d, logits_d, nullptr, s);
  });
}

tt2_status tt2_wn_cond_from_mels_dev(const float* mels_d, int ld_t, const int32_t* lengths_d, int B, int T_f,
                                     int num_mels, float lo, float hi, int clip, int normalize, float* cond_d,
                                     void* stream) {
  return guard([&] {
    TT2_CHECK(mels_d && lengths_d && cond_d, TT2_ERR_INVALID_ARG, "tt2_wn_cond_from_mels_dev: null argument");
    TT2_CHECK(B >= 1 && T_f >= 1 && num_mels >= 1 && ld_t >= 1, TT2_ERR_SHAPE_MISMATCH,
              "tt2_wn_cond_from_mels_dev: bad sizes");
    TT2_CHECK(hi > lo, TT2_ERR_INVALID_ARG, "tt2_wn_cond_from_mels_dev: empty output range");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_cond_from_mels, dim3(cdiv(T_f, 32), cdiv(num_mels, 32), B), dim3(256), 0, s, mels_d,
                       (long)ld_t, lengths_d, num_mels, T_f, lo, hi, clip, normalize, cond_d);
    TT2_HIP(hipGetLastError());
  });
}

tt2_status tt2_wn_noise(uint64_t seed, int T, int B, int nr_mix, int gaussian, float* u_mix, float* u_log) {
  return guard([&] {
    TT2_CHECK(u_log && (gaussian || u_mix), TT2_ERR_INVALID_ARG, "tt2_wn_noise: null argument");
    TT2_CHECK(T >= 1 && B >= 1 && (gaussian || (nr_mix >= 1 && nr_mix <= 14)), TT2_ERR_INVALID_ARG,
              "tt2_wn_noise: bad sizes");
    const long n = (long)T * B;
    const int nm = gaussian ? 0 : nr_mix;
    DevBuf dm, dl;
    if (nm) dm.alloc(sizeof(float) * n * nm);
    dl.alloc(sizeof(float) * n);
    hipLaunchKernelGGL(k_wn_noise, dim3((unsigned)std::min<long>((n + 255) / 256, 65535)), dim3(256), 0, 0, seed, n, B,
                       nm, gaussian, dm.as<float>(), dl.as<float>());
    TT2_HIP(hipGetLastError());
    if (nm) TT2_HIP(hipMemcpy(u_mix, dm.p, sizeof(float) * n * nm, hipMemcpyDeviceToHost));
    TT2_HIP(hipMemcpy(u_log, dl.p, sizeof(float) * n, hipMemcpyDeviceToHost));
  });
}

tt2_status tt2_mol_sample(const float* logits, const float* u_mix, const float* u_log, int n, int nr_mix,
                          float log_scale_min, float* x, int32_t* k) {
  return guard([&] {
    TT2_CHECK(logits && u_mix && u_log && x && k, TT2_ERR_INVALID_ARG, "tt2_mol_sample: null argument");
    TT2_CHECK(n >= 1 && nr_mix >= 1 && nr_mix <= 64, TT2_ERR_INVALID_ARG, "tt2_mol_sample: bad sizes");
    DevBuf dl, dm, du, dx, dk;
    dl.alloc(sizeof(float) * n * 3 * nr_mix);
    dm.alloc(sizeof(float) * n * nr_mix);
    du.alloc(sizeof(float) * n);
    dx.alloc(sizeof(float) * n);
    dk.alloc(sizeof(int) * n);
    TT2_HIP(hipMemcpy(dl.p, logits, sizeof(float) * n * 3 * nr_mix, hipMemcpyHostToDevice));
    TT2_HIP(hipMemcpy(dm.p, u_mix, sizeof(float) * n * nr_mix, hipMemcpyHostToDevice));
    TT2_HIP(hipMemcpy(du.p, u_log, sizeof(float) * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_mol_sample, dim3((n + 3) / 4), dim3(256), 0, 0, dl.as<float>(), dm.as<float>(), du.as<float>(),
                       n, nr_mix, log_scale_min, dx.as<float>(), dk.as<int>());
    TT2_HIP(hipGetLastError());
    TT2_HIP(hipMemcpy(x, dx.p, sizeof(float) * n, hipMemcpyDeviceToHost));
    TT2_HIP(hipMemcpy(k, dk.p, sizeof(int) * n, hipMemcpyDeviceToHost));
  });
}

}  // extern "C"
