// WaveNet MoL vocoder synthesis on MI355X (gfx950).
//
// Reference: code/wavenet_vocoder/models/wavenet.py (incremental :724-911, upsampling :782-803),
// modules.py (CausalConv1D incremental :273-303, ResidualConv1DGLU.step :471-521,
// ConvTranspose2D :736-770), mixture.py (sample_from_discretized_mix_logistic :76-107).
//
// Pipeline per call:
//   1. k_upsample × n_upsample   ConvTranspose2D(kernel (3,s), stride (1,s), 'same') + ReLU
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

namespace tt2 {

static const char* WP = "WaveNet_model/inference/";

// ConvTranspose2D 1→1 channel, kernel (KF, s), stride (1, s), 'same' (modules.py:736-770):
//   out[b][f][i*s+j] = relu(Σ_d in[b][f+pad-d][i] · K[d][j] + bias),  pad = (KF-1)/2
__global__ void k_upsample(const float* __restrict__ in, float* __restrict__ out, float* __restrict__ out_t,
                           const float* __restrict__ K, const float* __restrict__ bias, int B, int F, int Tin,
                           int s, int KF) {
  const long Tout = (long)Tin * s;
  const long n = (long)B * F * Tout;
  const int pad = (KF - 1) / 2;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int b = e / ((long)F * Tout);
    const long r = e - (long)b * F * Tout;
    const int f = r / Tout;
    const long to = r - (long)f * Tout;
    const int i = to / s, j = to - (long)i * s;
    float acc = 0.f;
    for (int d = 0; d < KF; ++d) {
      const int ff = f + pad - d;
      if (ff >= 0 && ff < F) acc += in[((long)b * F + ff) * Tin + i] * K[d * s + j];
    }
    const float y = fmaxf(acc + bias[0], 0.f);
    out[e] = y;
    if (out_t) out_t[((long)b * Tout + to) * F + f] = y;
  }
}

// Column order of the gated conv / cond outputs per quad q: {a_2q, a_2q+1, b_2q, b_2q+1}
// so the lane that reduces quad q can apply tanh(a)·σ(b) without a cross-lane exchange.
static inline int gate_col(int R, int q, int e) { return (e < 2 ? 2 * q + e : R + 2 * q + (e - 2)); }

constexpr int WN_THREADS = 256;

struct GenArgs {
  int B, T, L, stacks;
  const float* first_w; const float* first_b;      // [R], [R]
  const f32x4* conv_w;  // [L][24][256] float4 (R=64: quad q, k-slice ks -> tid = q*8+ks)
  const float* conv_b;  // [L][G] permuted
  const float* cond;    // [B][T][L][G] permuted (includes cond bias)
  const f32x4* so_w;    // [L][8][256] float4: [Ws|Wo][ks*8+k'][4q..4q+3]
  const float* so_b;    // [L][2R] = [bs | bo]
  const float* f1_w; const float* f1_b;  // [S][S], [S]
  const float* f2_w; const float* f2_b;  // [S][C], [C]
  int C;                // out_channels
  int legacy, res_legacy;
  float log_scale_min;
  const float* u_mix; const float* u_log;  // [T][B][nr], [T][B] or null
  uint64_t seed;
  const float* teacher;  // [B][T] or null
  float* wav; int* kout; float* logits;
};

__device__ __forceinline__ float gumbel_L(double u) { return (float)log(-log(u)); }

// R = 64, G = 128, S = 64 (BASELINE config 3).  256 threads = 4 waves, one per SIMD, so each
// lane may hold 512 VGPRs: the current and the next layer's weights (2 x 128 VGPRs) stay in
// registers and the next layer's stream is in flight while the current layer computes.
// Dilated conv:  tid = q*8 + ks -> output quad q (gate-permuted columns), k-slice ks of 24.
// Skip/out 1x1:  tid = q*8 + ks -> output quad q (q<16 skip, q>=16 out), k-slice ks of 8.
// Cross-slice sums are shuffle reductions over 8 lanes; two barriers per layer.
__global__ __launch_bounds__(WN_THREADS) void k_generate64(GenArgs a) {
  constexpr int R = 64, G = 128, S = 64, NT = WN_THREADS;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = tid >> 3, ks = tid & 7;
  const int L = a.L, per = L / a.stacks, LG = L * G;
  float* in = sm;            // [3R] conv input: taps t-2d, t-d, current x
  float* z = in + 3 * R;     // [R] gated activations
  float* skv = z + R;        // [S]
  float* h1 = skv + S;       // [S]
  float* lg = h1 + S;        // [32] logits
  float* misc = lg + 32;     // [16] misc[0] = next input sample
  float* cbuf = misc + 16;   // [L*G] conditioning of the current sample
  float* rings = cbuf + LG;  // per-layer rings of 2d+1 entries
  const f32x4* cond4 = reinterpret_cast<const f32x4*>(a.cond);
  f32x4* cbuf4 = reinterpret_cast<f32x4*>(cbuf);
  // head weights live in registers for the whole utterance
  const int q2 = tid >> 4, k2 = tid & 15;  // f1: 16 quads x 16 slices of 4 k
  f32x4 hw1[4];
  for (int e = 0; e < 4; ++e) hw1[e] = *reinterpret_cast<const f32x4*>(a.f1_w + (4 * k2 + e) * S + 4 * q2);
  const f32x4 hb1 = *reinterpret_cast<const f32x4*>(a.f1_b + 4 * q2);
  const int q3 = tid >> 5, k3 = tid & 31;  // f2: 8 quads (32 >= C columns) x 32 slices of 2 k
  float hw2[2][4], hb2[4];
  for (int e = 0; e < 4; ++e) {
    const int col = 4 * q3 + e;
    for (int kk = 0; kk < 2; ++kk) hw2[kk][e] = col < a.C ? a.f2_w[(2 * k3 + kk) * a.C + col] : 0.f;
    hb2[e] = col < a.C ? a.f2_b[col] : 0.f;
  }
  int ring_total = 0;
  for (int l = 0; l < L; ++l) ring_total += (2 * (1 << (l % per)) + 1) * R;
  for (int i = tid; i < ring_total; i += NT) rings[i] = 0.f;
  for (int i = tid; i < LG / 4; i += NT) cbuf4[i] = cond4[((long)b * a.T) * (LG / 4) + i];
  if (tid == 0) misc[0] = 0.f;  // initial input 0 for 'raw' (wavenet.py:437-445)
  const float SQH = 0.70710677f; // float32(np.sqrt(0.5))
  const f32x4* cw4 = a.conv_w;
  const f32x4* so4 = a.so_w;
  const f32x4* cb4 = reinterpret_cast<const f32x4*>(a.conv_b);
  const f32x4* sb4 = reinterpret_cast<const f32x4*>(a.so_b);
  f32x4 wc[24], ws[8];
#pragma unroll
  for (int kk = 0; kk < 24; ++kk) wc[kk] = cw4[kk * NT + tid];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) ws[kk] = so4[kk * NT + tid];
  __syncthreads();

  for (int t = 0; t < a.T; ++t) {
    // ---- prefetch: next sample's conditioning, this sample's MoL uniforms / teacher value ----
    constexpr int NCN = 3;  // ceil(L*G/4 / NT) for L <= 24
    f32x4 cn[NCN];
    const bool has_next = t + 1 < a.T;
#pragma unroll
    for (int i = 0; i < NCN; ++i) {
      const int idx = tid + i * NT;
      if (has_next && idx < LG / 4) cn[i] = cond4[((long)b * a.T + t + 1) * (LG / 4) + idx];
    }
    float um = 0.5f, ul = 0.5f, tv = 0.f;
    if (tid < 10)
      um = a.u_mix ? a.u_mix[((long)t * a.B + b) * 10 + tid]
                   : (float)u01_open(mix64(a.seed ^ mix64(((uint64_t)t * a.B + b) * 16 + tid)));
    if (tid == 0) {
      ul = a.u_log ? a.u_log[(long)t * a.B + b]
                   : (float)u01_open(mix64(a.seed ^ mix64(((uint64_t)t * a.B + b) * 16 + 15)));
      if (a.teacher) tv = a.teacher[(long)b * a.T + t];
    }
    // ---- first conv (Conv1D1x1, in=1) + layer-0 queue ----
    if (tid < R) {
      const float x0 = misc[0] * a.first_w[tid] + a.first_b[tid];
      const int Ld = 3;  // d = 1
      in[0 * R + tid] = rings[((t + 1) % Ld) * R + tid];      // x(t-2d)
      in[1 * R + tid] = rings[((t + Ld - 1) % Ld) * R + tid];  // x(t-d)
      in[2 * R + tid] = x0;
      rings[(t % Ld) * R + tid] = x0;
    }
    f32x4 skips = {0.f, 0.f, 0.f, 0.f};
    int roff = 0;
    __syncthreads();
    for (int l = 0; l < L; ++l) {
      const int d = 1 << (l % per), Ld = 2 * d + 1;
      const int ln = (l + 1 == L) ? 0 : l + 1;  // prefetch wraps to layer 0 of the next sample
      f32x4 nwc[24], nws[8];
#pragma unroll
      for (int kk = 0; kk < 24; ++kk) nwc[kk] = cw4[((long)ln * 24 + kk) * NT + tid];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) nws[kk] = so4[((long)ln * 8 + kk) * NT + tid];
      f32x4 cb = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
      if (ks == 0) {
        cb = cb4[l * (G / 4) + q];
        sb = sb4[l * (G / 4) + q];
      }
      // dilated conv GEMV over the 3 queue taps (modules.py:283-297)
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const f32x4* ip4 = reinterpret_cast<const f32x4*>(in + ks * 24);
#pragma unroll
      for (int k4 = 0; k4 < 6; ++k4) {
        const f32x4 xv = ip4[k4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x4 w = wc[k4 * 4 + e];
          acc[0] += xv[e] * w[0]; acc[1] += xv[e] * w[1]; acc[2] += xv[e] * w[2]; acc[3] += xv[e] * w[3];
        }
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        acc[0] += __shfl_xor(acc[0], o); acc[1] += __shfl_xor(acc[1], o);
        acc[2] += __shfl_xor(acc[2], o); acc[3] += __shfl_xor(acc[3], o);
      }
      if (ks == 0) {  // (conv + b) + (cond·W + b_c), gated tanh·σ (modules.py:494-510)
        const f32x4 cd = cbuf4[l * (G / 4) + q];
        const float av0 = (acc[0] + cb[0]) + cd[0];
        const float av1 = (acc[1] + cb[1]) + cd[1];
        const float bv0 = (acc[2] + cb[2]) + cd[2];
        const float bv1 = (acc[3] + cb[3]) + cd[3];
        z[2 * q] = tanhf(av0) * sigm(bv0);
        z[2 * q + 1] = tanhf(av1) * sigm(bv1);
      }
      __syncthreads();
      // skip / out 1x1 (modules.py:512-520)
      f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};
      const f32x4* zp4 = reinterpret_cast<const f32x4*>(z + ks * 8);
#pragma unroll
      for (int k4 = 0; k4 < 2; ++k4) {
        const f32x4 zv = zp4[k4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x4 w = ws[k4 * 4 + e];
          acc2[0] += zv[e] * w[0]; acc2[1] += zv[e] * w[1]; acc2[2] += zv[e] * w[2]; acc2[3] += zv[e] * w[3];
        }
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        acc2[0] += __shfl_xor(acc2[0], o); acc2[1] += __shfl_xor(acc2[1], o);
        acc2[2] += __shfl_xor(acc2[2], o); acc2[3] += __shfl_xor(acc2[3], o);
      }
      if (ks == 0) {
        if (q < 16) {  // skip connection sum (wavenet.py:833-836)
          f32x4 sv;
          for (int e = 0; e < 4; ++e) sv[e] = acc2[e] + sb[e];
          if (l == 0) skips = sv;
          else if (a.legacy) for (int e = 0; e < 4; ++e) skips[e] = (skips[e] + sv[e]) * SQH;
          else for (int e = 0; e < 4; ++e) skips[e] = skips[e] + sv[e];
        } else if (l + 1 < L) {  // residual output -> next layer's input and queue
          const int j = 4 * (q - 16);
          const int dn = 1 << ((l + 1) % per), Ln = 2 * dn + 1;
          float* ringn = rings + roff + Ld * R;
          for (int e = 0; e < 4; ++e) {
            float xo = (acc2[e] + sb[e]) + in[2 * R + j + e];
            if (a.res_legacy) xo = xo * SQH;
            in[2 * R + j + e] = xo;
            ringn[(t % Ln) * R + j + e] = xo;
            in[0 * R + j + e] = ringn[((t + 1) % Ln) * R + j + e];
            in[1 * R + j + e] = ringn[((t + Ln - dn) % Ln) * R + j + e];
          }
        }
      }
      roff += Ld * R;
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < 24; ++kk) wc[kk] = nwc[kk];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) ws[kk] = nws[kk];
    }
    // next sample's conditioning -> LDS (every read of this sample's cbuf is behind a barrier)
#pragma unroll
    for (int i = 0; i < NCN; ++i) {
      const int idx = tid + i * NT;
      if (has_next && idx < LG / 4) cbuf4[idx] = cn[i];
    }
    // ---- head: ReLU -> 1x1 -> ReLU -> 1x1 (wavenet.py:840-844) ----
    if (ks == 0 && q < 16)
      for (int e = 0; e < 4; ++e) skv[4 * q + e] = fmaxf(skips[e], 0.f);
    __syncthreads();
    {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const f32x4 xv = reinterpret_cast<const f32x4*>(skv)[k2];
      for (int e = 0; e < 4; ++e) {
        acc[0] += xv[e] * hw1[e][0]; acc[1] += xv[e] * hw1[e][1];
        acc[2] += xv[e] * hw1[e][2]; acc[3] += xv[e] * hw1[e][3];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        acc[0] += __shfl_xor(acc[0], o); acc[1] += __shfl_xor(acc[1], o);
        acc[2] += __shfl_xor(acc[2], o); acc[3] += __shfl_xor(acc[3], o);
      }
      if (k2 == 0)
        for (int e = 0; e < 4; ++e) h1[4 * q2 + e] = fmaxf(acc[e] + hb1[e], 0.f);
    }
    __syncthreads();
    {
      float acc[4];
      const float x0 = h1[2 * k3], x1 = h1[2 * k3 + 1];
      for (int e = 0; e < 4; ++e) acc[e] = x0 * hw2[0][e] + x1 * hw2[1][e];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1)
        for (int e = 0; e < 4; ++e) acc[e] += __shfl_xor(acc[e], o);
      if (k3 == 0)
        for (int e = 0; e < 4; ++e) {
          const int col = 4 * q3 + e;
          if (col < a.C) {
            lg[col] = acc[e] + hb2[e];
            if (a.logits) a.logits[((long)b * a.T + t) * a.C + col] = lg[col];
          }
        }
    }
    __syncthreads();
    // ---- MoL sampler (mixture.py:76-107), wave 0 ----
    if (tid < 64) {
      const int nr = a.C / 3;
      float temp = -INFINITY;
      int idx = lane;
      if (lane < nr) temp = lg[lane] - gumbel_L((double)um);
      for (int o = 32; o > 0; o >>= 1) {
        const float ot = __shfl_xor(temp, o);
        const int oi = __shfl_xor(idx, o);
        if (ot > temp || (ot == temp && oi < idx)) { temp = ot; idx = oi; }
      }
      if (lane == 0) {
        const float mean = lg[nr + idx];
        const float ls = fmaxf(lg[2 * nr + idx], a.log_scale_min);
        const double uu = (double)ul;
        const float noise = (float)(log(uu) - log(1.0 - uu));
        float x = mean + expf(ls) * noise;
        x = fminf(fmaxf(x, -1.f), 1.f);
        a.wav[(long)b * a.T + t] = x;
        if (a.kout) a.kout[(long)b * a.T + t] = idx;
        misc[0] = a.teacher ? tv : x;  // wavenet.py:876-878 test_inputs override
      }
    }
    __syncthreads();
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
  tt2::DevBuf up_k[8], up_b[8];
  tt2::DevBuf cin_d, up_a, up_b_buf, c_up_t, cond, umix, ulog, teacher, wav, kout, logits;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool timed = false;
};

namespace tt2 {

static void wupload(DevBuf& d, const std::vector<float>& h) {
  d.alloc(h.size() * sizeof(float));
  TT2_HIP(hipMemcpy(d.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
}

static void wn_finalize(tt2_wn_ctx* c) {
  const WeightMap& wm = c->host;
  const std::string P(WP);
  const int R = c->R, G = c->G, S = c->S, L = c->L, C = c->C, cin = c->cin, kw = c->cfg.kernel_size;
  TT2_HIP(hipSetDevice(c->dev));
  wupload(c->first_w, need(wm, P + "input_convolution/kernel", {1, 1, R}).data);
  wupload(c->first_b, need(wm, P + "input_convolution/bias", {R}).data);
  constexpr int CK = 3 * 64 / (WN_THREADS / 32);  // conv k's per slice (24)
  constexpr int SK = 64 / (WN_THREADS / 32);      // skip/out k's per slice (8)
  std::vector<float> cw((size_t)L * CK * WN_THREADS * 4), cb((size_t)L * G), condw((size_t)cin * L * G),
      condb((size_t)L * G), sow((size_t)L * SK * WN_THREADS * 4), sob((size_t)L * 2 * R);
  for (int l = 0; l < L; ++l) {
    const std::string s = P + "ResidualConv1DGLU_" + std::to_string(l) + "/";
    const std::string ln = "_ResidualConv1DGLU_" + std::to_string(l) + "/";
    const auto& k = need(wm, s + "residual_block_causal_conv" + ln + "kernel", {kw, R, G});
    const auto& bb = need(wm, s + "residual_block_causal_conv" + ln + "bias", {G});
    const auto& kc = need(wm, s + "residual_block_cin_conv" + ln + "kernel", {1, cin, G});
    const auto& bc = need(wm, s + "residual_block_cin_conv" + ln + "bias", {G});
    const auto& ksk = need(wm, s + "residual_block_skip_conv" + ln + "kernel", {1, G / 2, S});
    const auto& bsk = need(wm, s + "residual_block_skip_conv" + ln + "bias", {S});
    const auto& ko = need(wm, s + "residual_block_out_conv" + ln + "kernel", {1, G / 2, R});
    const auto& bo = need(wm, s + "residual_block_out_conv" + ln + "bias", {R});
    for (int tid = 0; tid < WN_THREADS; ++tid) {
      const int q = tid / (WN_THREADS / 32), ks = tid % (WN_THREADS / 32);
      for (int kk = 0; kk < CK; ++kk) {
        const int kidx = ks * CK + kk;  // row of the linearized [kw*R, G] weight
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
        condb[(size_t)l * G + dst] = bc.data[src];
        for (int i = 0; i < cin; ++i) condw[(size_t)i * L * G + l * G + dst] = kc.data[(size_t)i * G + src];
      }
    for (int j = 0; j < S; ++j) sob[(size_t)l * 2 * R + j] = bsk.data[j];
    for (int j = 0; j < R; ++j) sob[(size_t)l * 2 * R + S + j] = bo.data[j];
  }
  wupload(c->conv_w, cw);
  wupload(c->conv_b, cb);
  wupload(c->cond_w, condw);
  wupload(c->cond_b, condb);
  wupload(c->so_w, sow);
  wupload(c->so_b, sob);
  wupload(c->f1_w, need(wm, P + "skip_convolutions/final_convolution_1/kernel", {1, S, S}).data);
  wupload(c->f1_b, need(wm, P + "skip_convolutions/final_convolution_1/bias", {S}).data);
  wupload(c->f2_w, need(wm, P + "skip_convolutions/final_convolution_2/kernel", {1, S, C}).data);
  wupload(c->f2_b, need(wm, P + "skip_convolutions/final_convolution_2/bias", {C}).data);
  for (int i = 0; i < c->cfg.n_upsample; ++i) {
    const std::string sc = P + "local_conditioning_upsampling_" + std::to_string(i + 1) + "/ConvTranspose2D_layer_" +
                           std::to_string(i) + "/";
    const int s = c->cfg.upsample_scales[i], kf = c->cfg.freq_axis_kernel_size;
    wupload(c->up_k[i], need(wm, sc + "kernel", {kf, s, 1, 1}).data);
    wupload(c->up_b[i], need(wm, sc + "bias", {1}).data);
  }
  c->finalized = true;
}

static size_t gen_lds_bytes(const tt2_wn_ctx* c) {
  const int per = c->L / c->cfg.stacks;
  long ring = 0;
  for (int l = 0; l < c->L; ++l) ring += (2 * (1 << (l % per)) + 1) * c->R;
  return sizeof(float) * (3 * c->R + c->R + c->S + c->S + 32 + 16 + (long)c->L * c->G + ring);
}

static void wn_generate_dev(tt2_wn_ctx* c, const float* cond_in, int B, int T_f, const float* umix_d,
                            const float* ulog_d, uint64_t seed, const float* teacher_d, float* wav_d, int* k_d,
                            float* logits_d, float* upsampled_d, hipStream_t s) {
  TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_wn_finalize not called");
  TT2_CHECK(B >= 1 && B <= c->cfg.max_batch, TT2_ERR_SHAPE_MISMATCH, "batch exceeds capacity");
  const long T = (long)T_f * c->hop;
  TT2_CHECK(T_f >= 1 && T <= c->cfg.max_samples, TT2_ERR_SHAPE_MISMATCH, "synthesis length exceeds capacity");
  const int F = c->cin;
  // upsampling network: [B][F][T_f] -> [B][F][T]
  c->up_a.alloc(sizeof(float) * B * F * T);
  c->up_b_buf.alloc(sizeof(float) * B * F * T);
  c->c_up_t.alloc(sizeof(float) * B * T * F);
  TT2_HIP(hipEventRecord(c->ev[0], s));
  const float* src = cond_in;  // [B][F][T_f] channels-first
  long Tcur = T_f;
  float* bufs[2] = {c->up_a.as<float>(), c->up_b_buf.as<float>()};
  for (int i = 0; i < c->cfg.n_upsample; ++i) {
    const int sc = c->cfg.upsample_scales[i];
    const bool last = i + 1 == c->cfg.n_upsample;
    float* dst = (last && upsampled_d) ? upsampled_d : bufs[i & 1];
    const long n = (long)B * F * Tcur * sc;
    const int grid = (int)std::min<long>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(k_upsample, dim3(grid), dim3(256), 0, s, src, dst, last ? c->c_up_t.as<float>() : nullptr,
                       c->up_k[i].as<float>(), c->up_b[i].as<float>(), B, F, (int)Tcur, sc,
                       c->cfg.freq_axis_kernel_size);
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
  gemm(g, s);
  TT2_HIP(hipEventRecord(c->ev[2], s));
  GenArgs a;
  a.B = B; a.T = (int)T; a.L = c->L; a.stacks = c->cfg.stacks;
  a.first_w = c->first_w.as<float>(); a.first_b = c->first_b.as<float>();
  a.conv_w = c->conv_w.as<f32x4>(); a.conv_b = c->conv_b.as<float>(); a.cond = c->cond.as<float>();
  a.so_w = c->so_w.as<f32x4>(); a.so_b = c->so_b.as<float>();
  a.f1_w = c->f1_w.as<float>(); a.f1_b = c->f1_b.as<float>(); a.f2_w = c->f2_w.as<float>(); a.f2_b = c->f2_b.as<float>();
  a.C = c->C; a.legacy = c->cfg.legacy; a.res_legacy = c->cfg.residual_legacy; a.log_scale_min = c->cfg.log_scale_min;
  a.u_mix = umix_d; a.u_log = ulog_d; a.seed = seed; a.teacher = teacher_d;
  a.wav = wav_d; a.kout = k_d; a.logits = logits_d;
  const size_t shm = gen_lds_bytes(c);
  hipLaunchKernelGGL(k_generate64, dim3(B), dim3(WN_THREADS), shm, s, a);
  TT2_HIP(hipGetLastError());
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
}

tt2_status tt2_wn_create(const tt2_wn_config* cfg, int hip_device, tt2_wn_ctx** out) {
  return guard([&] {
    TT2_CHECK(cfg && out, TT2_ERR_INVALID_ARG, "tt2_wn_create: null argument");
    *out = nullptr;
    int ndev = 0;
    TT2_HIP(hipGetDeviceCount(&ndev));
    TT2_CHECK(hip_device >= 0 && hip_device < ndev, TT2_ERR_INVALID_ARG, "tt2_wn_create: bad device index");
    TT2_CHECK(cfg->residual_channels == 64 && cfg->gate_channels == 128 && cfg->skip_out_channels == 64,
              TT2_ERR_INVALID_ARG,
              "this build's generation kernel is specialised for R=64, G=128, S=64 (BASELINE config 3)");
    TT2_CHECK(cfg->kernel_size == 3, TT2_ERR_INVALID_ARG, "kernel_size must be 3");
    TT2_CHECK(cfg->out_channels % 3 == 0 && cfg->out_channels <= 30 && cfg->out_channels >= 3, TT2_ERR_INVALID_ARG,
              "MoL head needs out_channels = 3*nr_mix <= 30");
    TT2_CHECK(cfg->layers >= 1 && cfg->stacks >= 1 && cfg->layers % cfg->stacks == 0, TT2_ERR_INVALID_ARG,
              "layers % stacks != 0");
    TT2_CHECK(cfg->layers * cfg->gate_channels / 4 <= 3 * WN_THREADS, TT2_ERR_INVALID_ARG,
              "conditioning row of one sample exceeds the prefetch registers (layers*G <= 3072)");
    TT2_CHECK(cfg->cin_channels >= 1 && cfg->cin_channels <= 128, TT2_ERR_INVALID_ARG, "cin_channels out of range");
    TT2_CHECK(cfg->n_upsample >= 1 && cfg->n_upsample <= 8, TT2_ERR_INVALID_ARG, "n_upsample out of range");
    TT2_CHECK(cfg->max_batch >= 1 && cfg->max_samples >= 1, TT2_ERR_INVALID_ARG, "capacities must be >= 1");
    auto c = std::make_unique<tt2_wn_ctx>();
    c->cfg = *cfg;
    c->dev = hip_device;
    c->R = cfg->residual_channels; c->G = cfg->gate_channels; c->S = cfg->skip_out_channels;
    c->L = cfg->layers; c->C = cfg->out_channels; c->cin = cfg->cin_channels;
    c->hop = 1;
    for (int i = 0; i < cfg->n_upsample; ++i) c->hop *= cfg->upsample_scales[i];
    TT2_HIP(hipSetDevice(hip_device));
    TT2_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (auto& e : c->ev) TT2_HIP(hipEventCreate(&e));
    const size_t shm = gen_lds_bytes(c.get());
    TT2_CHECK(shm <= 160 * 1024, TT2_ERR_INVALID_ARG, "queue rings exceed the 160 KiB LDS of a CU");
    TT2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_generate64),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    *out = c.release();
  });
}

void tt2_wn_destroy(tt2_wn_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  delete c;
}

tt2_status tt2_wn_last_timings(tt2_wn_ctx* c, float* ms3) {
  return guard([&] {
    TT2_CHECK(c && ms3, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->timed, TT2_ERR_STATE, "no generate call yet");
    TT2_HIP(hipEventSynchronize(c->ev[3]));
    for (int i = 0; i < 3; ++i) TT2_HIP(hipEventElapsedTime(&ms3[i], c->ev[i], c->ev[i + 1]));
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
    const int F = c->cin, nr = c->C / 3;
    // host layout [B][T_f][F] -> device channels-first [B][F][T_f]
    std::vector<float> cf((size_t)B * F * T_f);
    for (int b = 0; b < B; ++b)
      for (int t = 0; t < T_f; ++t)
        for (int f = 0; f < F; ++f) cf[((size_t)b * F + f) * T_f + t] = cond[((size_t)b * T_f + t) * F + f];
    c->cin_d.alloc(cf.size() * sizeof(float));
    TT2_HIP(hipMemcpyAsync(c->cin_d.p, cf.data(), cf.size() * sizeof(float), hipMemcpyHostToDevice, s));
    const float *um = nullptr, *ul = nullptr, *tg = nullptr;
    if (u_mix) {
      c->umix.alloc(sizeof(float) * T * B * nr);
      TT2_HIP(hipMemcpyAsync(c->umix.p, u_mix, sizeof(float) * T * B * nr, hipMemcpyHostToDevice, s));
      um = c->umix.as<float>();
    }
    if (u_log) {
      c->ulog.alloc(sizeof(float) * T * B);
      TT2_HIP(hipMemcpyAsync(c->ulog.p, u_log, sizeof(float) * T * B, hipMemcpyHostToDevice, s));
      ul = c->ulog.as<float>();
    }
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
