// WaveNet synthesis for input_type 'mulaw-quantize' (wavenet_q.h): the WaveNet.incremental loop of
// wavenet.py:724-911 with one-hot inputs (wavenet.py:433-446) and the softmax head sampled by
// tf.multinomial (softmax=False, quantize=True: :861-867), then inv_mulaw_quantize (:450-452).
//
// One work-group (16 waves) per utterance runs every layer of a sample: the per-layer products are
// GEMVs whose weights stream from L2 / MALL (the fused layer-resident generators of wavenet.hip /
// wavenet_wide.hip carry the scalar-input heads; this path covers the one-hot input and the
// Q-class head at the reference's default widths, not at their speed).  Every sample:
//   x = first_w[k_{t-1}] + first_b                       (first_conv of a one-hot row)
//   per layer: queue x; h = [x(t-2d) | x(t-d) | x]·W + b + cond_t; z = tanh(h_a)·σ(h_b);
//              [skip | out] = z·[Ws | Wo] + b; skips += skip; x = out + x   (legacy scalings)
//   logits = relu(relu(skips)·F1 + b1)·F2 + b2
//   k = first class whose running Σ exp(logit - max) (float64) exceeds u·total  (TF's multinomial)
#include "wavenet_q.h"

namespace tt2 {

long wq_ring_floats(int R, int L, int per) {
  long n = 0;
  for (int l = 0; l < L; ++l) n += (2L * (1 << (l % per)) + 1) * R;
  return n;
}

size_t wq_lds_bytes(int R, int G, int S, int Q) {
  // xin[R] vt[3R] part[4 NT] hg[G] z[R] skip[S] hb[S] lg[Q] pref[64 doubles] scalars[16]
  return sizeof(float) * ((size_t)R + 3 * R + 4 * WQ_THREADS + G + R + S + S + Q + 128 + 16);
}

typedef float wq_f4 __attribute__((ext_vector_type(4)));

// y = Σ_{k<K} v[k]·W[k·ld + c] for columns c < N (N, ld multiples of 4): a thread owns a column quad
// (16-byte weight loads) of one of NKS = NT / (N / 4) k-slices, 16 loads in flight per batch;
// partials summed in slice order by the column's thread (returned for tid < N; every thread takes
// the barriers)
__device__ __forceinline__ float wq_gemv(const float* v, const float* __restrict__ W, long ld, int K, int N,
                                         float* part) {
  const int tid = threadIdx.x, nq = N / 4, nks = max(1, WQ_THREADS / nq);
  const int cq = tid % nq, ks = tid / nq;
  if (ks < nks) {
    const int k0 = ks * K / nks, k1 = (ks + 1) * K / nks;
    const wq_f4* w4 = reinterpret_cast<const wq_f4*>(W) + cq;
    const long ld4 = ld / 4;
    wq_f4 acc = {0.f, 0.f, 0.f, 0.f};
    int k = k0;
    for (; k + 16 <= k1; k += 16) {
      wq_f4 wv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) wv[i] = w4[(long)(k + i) * ld4];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc += v[k + i] * wv[i];
    }
    for (; k < k1; ++k) acc += v[k] * w4[(long)k * ld4];
    *reinterpret_cast<wq_f4*>(part + ks * N + 4 * cq) = acc;
  }
  __syncthreads();
  float y = 0.f;
  if (tid < N)
    for (int s = 0; s < nks; ++s) y += part[s * N + tid];
  __syncthreads();
  return y;
}

__device__ __forceinline__ float wq_sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ __launch_bounds__(WQ_THREADS, 1) void k_generate_q(QGenArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int R = a.R, G = a.G, S = a.S, Q = a.Q, L = a.L;
  float* xin = sm;              // [R]
  float* vt = xin + R;          // [3R] taps | x; the head's relu input
  float* part = vt + 3 * R;     // [NT]
  float* hg = part + 4 * WQ_THREADS;  // [G]
  float* z = hg + G;            // [R]
  float* sk = z + R;            // [S] skip sum
  float* hb = sk + S;           // [S]
  float* lg = hb + S;           // [Q]
  double* pref = reinterpret_cast<double*>(lg + Q + ((Q & 1) ? 1 : 0));  // [64] chunk prefixes
  int* kbuf = reinterpret_cast<int*>(pref + 64);                           // [1] drawn class
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float SQH = 0.70710677f;  // float32(np.sqrt(0.5))
  float* const ring = a.rings + (long)b * a.ring_floats;
  int kprev = a.k0;
  for (int t = 0; t < a.T; ++t) {
    // ---- x = first_conv(one_hot(k_{t-1}))
    for (int r = tid; r < R; r += WQ_THREADS) xin[r] = a.first_w[(long)kprev * R + r] + a.first_b[r];
    for (int c = tid; c < S; c += WQ_THREADS) sk[c] = 0.f;
    __syncthreads();
    long ro = 0;
    for (int l = 0; l < L; ++l) {
      const int d = 1 << (l % a.per), len = 2 * d + 1;
      float* q = ring + ro;
      // queue x(t) (slot t mod len); the taps x(t-2d), x(t-d) sit in slots (t+1), (t-d) mod len
      const int s0 = (t + 1) % len, s1 = (t + len - d % len) % len, sw = t % len;
      for (int r = tid; r < R; r += WQ_THREADS) {
        vt[r] = q[(long)s0 * R + r];
        vt[R + r] = q[(long)s1 * R + r];
        vt[2 * R + r] = xin[r];
      }
      __syncthreads();
      for (int r = tid; r < R; r += WQ_THREADS) q[(long)sw * R + r] = xin[r];
      // gates: h = taps·W + b + cond
      const float hv = wq_gemv(vt, a.conv_w + (long)l * 3 * R * G, G, 3 * R, G, part);
      if (tid < G)
        hg[tid] = hv + a.conv_b[(long)l * G + tid] + (a.cond ? a.cond[(((long)b * a.T + t) * L + l) * G + tid] : 0.f);
      __syncthreads();
      for (int j = tid; j < R; j += WQ_THREADS) z[j] = tanhf(hg[j]) * wq_sigm(hg[R + j]);
      __syncthreads();
      // [skip | out] = z·[Ws | Wo] + b
      const float ov = wq_gemv(z, a.so_w + (long)l * R * (S + R), S + R, R, S + R, part);
      if (tid < S) {
        const float v = ov + a.so_b[(long)l * (S + R) + tid];
        sk[tid] = l == 0 ? v : (a.legacy ? (sk[tid] + v) * SQH : sk[tid] + v);
      } else if (tid < S + R) {
        const int r = tid - S;
        const float v = ov + a.so_b[(long)l * (S + R) + tid];
        hg[r] = a.res_legacy ? (v + xin[r]) * SQH : v + xin[r];  // hg: scratch for the next x
      }
      __syncthreads();
      for (int r = tid; r < R; r += WQ_THREADS) xin[r] = hg[r];
      __syncthreads();
      ro += (long)len * R;
    }
    // ---- head: relu -> 1x1 -> relu -> 1x1 (wavenet.py:840-844)
    for (int c = tid; c < S; c += WQ_THREADS) vt[c] = fmaxf(sk[c], 0.f);
    __syncthreads();
    const float h1 = wq_gemv(vt, a.f1_w, S, S, S, part);
    if (tid < S) hb[tid] = fmaxf(h1 + a.f1_b[tid], 0.f);
    __syncthreads();
    const float lv = wq_gemv(hb, a.f2_w, Q, S, Q, part);
    if (tid < Q) {
      const float x = lv + a.f2_b[tid];
      lg[tid] = x;
      if (a.logits) a.logits[((long)b * a.T + t) * Q + tid] = x;
    }
    __syncthreads();
    // ---- tf.multinomial: wave 0, lane i owns the classes [cq i, cq i + cq)
    if (wave == 0) {
      const int cq = (Q + 63) / 64, c0 = lane * cq, c1 = min(Q, c0 + cq);
      float mx = -INFINITY;
      for (int c = c0; c < c1; ++c)
        if (isfinite(lg[c])) mx = fmaxf(mx, lg[c]);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const double m = (double)mx;
      double run = 0.0;
      for (int c = c0; c < c1; ++c)
        if (isfinite(lg[c])) run += exp((double)lg[c] - m);
      // exclusive prefix of the chunk totals in lane order
      double ex = 0.0, tot = 0.0;
      for (int i = 0; i < 64; ++i) {
        const double v = __shfl(run, i, 64);
        if (i < lane) ex += v;
        tot += v;
      }
      const float u = a.u ? a.u[(long)t * a.Bg + b] : wn_uniform(a.seed, t, a.Bg, b, 0);
      const double target = (double)u * tot;
      // first class whose cdf exceeds the target (std::upper_bound)
      double cdf = ex;
      int found = -1;
      for (int c = c0; c < c1; ++c) {
        if (isfinite(lg[c])) cdf += exp((double)lg[c] - m);
        if (found < 0 && cdf > target) found = c;
      }
      // the lowest lane with a hit owns the draw
      const unsigned long long hit = __ballot(found >= 0);
      const int owner = hit ? __ffsll((long long)hit) - 1 : -1;
      const int kf = __shfl(found, owner < 0 ? 0 : owner, 64);
      if (lane == 0) kbuf[0] = owner < 0 ? Q - 1 : kf;
    }
    __syncthreads();
    const int k = kbuf[0];
    if (tid == 0) {
      const float y = 2.f * (float)k / 255.f - 1.f;  // util.inv_mulaw_quantize, mu = 255 (util.py:105-129)
      const float ay = fabsf(y);
      const float w = (y > 0.f ? 1.f : (y < 0.f ? -1.f : 0.f)) * (1.f / 255.f) * (powf(256.f, ay) - 1.f);
      a.wav[(long)b * a.T + t] = w;
      if (a.kout) a.kout[(long)b * a.T + t] = k;
    }
    // teacher classes are validated on the host for tt2_wn_generate*; device-side teachers
    // (tt2_wn_generate_dev) are clamped so a bad class cannot index past the first conv's rows
    kprev = a.teacher ? min(max((int)a.teacher[(long)b * a.T + t], 0), a.Q - 1) : k;
    __syncthreads();
  }
}

void wq_launch(const QGenArgs& a, hipStream_t s) {
  const size_t shm = wq_lds_bytes(a.R, a.G, a.S, a.Q);
  hipLaunchKernelGGL(k_generate_q, dim3(a.Bg), dim3(WQ_THREADS), shm, s, a);
  TT2_HIP(hipGetLastError());
}

}  // namespace tt2
