// Griffin-Lim vocoder on MI355X (gfx950): the reference's GPU variant, GL_on_GPU = True
// (code/hparams.py:135), used by tacotron/synthesizer.py:152-160,201-206 to write eval wavs:
//   datasets/audio.py:131-143  inv_{mel,linear}_spectrogram_tensorflow
//     D = _denormalize(x)                                  (audio.py:283-296)
//     S = (10^((D + ref_level_db) / 20))^(1/magnitude_power)
//     S = max(1e-10, S · pinv(mel_basis)^T)                (_mel_to_linear_tensorflow :237-241; mel only)
//     y = _griffin_lim_tensorflow(S^power)                 (:163-176)
//   _griffin_lim_tensorflow: y = inverse_stft(S + 0j); repeat griffin_lim_iters times:
//     est = stft(y); angles = est / max(1e-8, |est|); y = inverse_stft(S · angles)
//   with TF 1.x tf.contrib.signal semantics: frames of win_size samples every hop samples
//   (pad_end=False), periodic Hann window of win_size, rfft zero-padded to n_fft; inverse_stft =
//   irfft(n_fft)[:win_size] · window, then overlap-add.
//
// Kernels (one work-group of 256 threads per frame; the n_fft-point transform runs in LDS):
//   k_gl_amp     mel/linear frame -> amplitude A = (10^((D+ref)/20))^(1/mp)          elementwise
//   k_gl_spec    S[t][f] = max(1e-10, Σ_m A[t][m] · IB[f][m])^power  (mel) / A^power (linear)
//   k_gl_istft   X = S · angle (angle = 1 before the first iteration) -> irfft -> window ->
//                frame buffer Fr[t][0..win)
//   k_gl_stft    overlap-add gather of the frame's samples from Fr (every frame overlapping it),
//                window, rfft, angle = est / max(1e-8, |est|)
//   k_gl_ola     final overlap-add into the waveform [(T-1)·hop + win]
// All fp32; twiddles computed on the host in double.  HBM traffic per iteration is
// ~T·(3·(n_fft/2+1) + 2·win)·4 bytes (≈ 30 MB at T = 1000): the iteration is latency-bound by its
// two launches, not by bandwidth.
#include <hip/hip_runtime.h>

#include <cmath>
#include <memory>
#include <vector>

#include "common.h"

namespace tt2 {

constexpr int GL_NT = 256;
constexpr int GL_MAX_FFT = 4096;

// In-place radix-2 DIT FFT of n = 2^lg points in LDS (input in bit-reversed order), twiddles
// tw[k] = exp(-2πik/n), k < n/2 (sign flipped for the inverse).
__device__ __forceinline__ void gl_fft(float2* x, const float2* tw, int n, int lg, bool inverse) {
  for (int s = 1; s <= lg; ++s) {
    const int half = 1 << (s - 1);
    const int tstride = n >> s;
    for (int b = threadIdx.x; b < n / 2; b += GL_NT) {
      const int pos = b & (half - 1);
      const int i = ((b >> (s - 1)) << s) + pos;
      const int j = i + half;
      float2 w = tw[pos * tstride];
      if (inverse) w.y = -w.y;
      const float2 xj = x[j], xi = x[i];
      const float2 t = make_float2(w.x * xj.x - w.y * xj.y, w.x * xj.y + w.y * xj.x);
      x[j] = make_float2(xi.x - t.x, xi.y - t.y);
      x[i] = make_float2(xi.x + t.x, xi.y + t.y);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ int gl_brev(int i, int lg) { return (int)(__brev((unsigned)i) >> (32 - lg)); }

// periodic Hann window (tf.contrib.signal.hann_window(periodic=True)): 0.5 - 0.5 cos(2πn/N)
__device__ __forceinline__ float gl_hann(const float* win, int n) { return win[n]; }

// amplitude of one normalised frame value: _denormalize (audio.py:283-296) + db_to_amp + 1/mp
struct GlNorm {
  float max_abs, min_db, ref_db, inv_mp;
  int symmetric, clip;
};
__device__ __forceinline__ float gl_amp(float d, const GlNorm& n) {
  float D;
  if (n.symmetric) {
    const float x = n.clip ? fminf(fmaxf(d, -n.max_abs), n.max_abs) : d;
    D = ((x + n.max_abs) * -n.min_db / (2.f * n.max_abs)) + n.min_db;
  } else {
    const float x = n.clip ? fminf(fmaxf(d, 0.f), n.max_abs) : d;
    D = (x * -n.min_db / n.max_abs) + n.min_db;
  }
  const float a = powf(10.f, (D + n.ref_db) * 0.05f);
  return powf(a, n.inv_mp);
}

__global__ void k_gl_amp(const float* __restrict__ x, long n, GlNorm nm, float* __restrict__ a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    a[i] = gl_amp(x[i], nm);
}

// S[t][f] = max(1e-10, Σ_m A[t][m] · IB[f][m])^power (mel, M > 0) or A[t][f]^power (linear, M == 0).
// Block = 256 frequencies of one frame; the frame's M amplitudes are staged in LDS.
__global__ __launch_bounds__(GL_NT) void k_gl_spec(const float* __restrict__ A, const float* __restrict__ IB, int M,
                                                   int F, float power, float* __restrict__ S) {
  __shared__ float am[256];
  const int t = blockIdx.y, f = blockIdx.x * GL_NT + threadIdx.x;
  if (M > 0) {
    for (int m = threadIdx.x; m < M; m += GL_NT) am[m] = A[(long)t * M + m];
    __syncthreads();
    if (f < F) {
      float s = 0.f;
      const float* ib = IB + (long)f * M;
      for (int m = 0; m < M; ++m) s += am[m] * ib[m];
      S[(long)t * F + f] = powf(fmaxf(1e-10f, s), power);
    }
  } else if (f < F) {
    S[(long)t * F + f] = powf(A[(long)t * F + f], power);
  }
}

// One frame: X[k] = S[k]·angle[k] (angle = 1 when ang == null), k <= n/2, Hermitian-extended;
// irfft; first `win` samples times the window -> Fr[t][·].
__global__ __launch_bounds__(GL_NT) void k_gl_istft(const float* __restrict__ S, const float2* __restrict__ ang,
                                                    const float2* __restrict__ tw_g, const float* __restrict__ win_g,
                                                    int n, int lg, int win, float* __restrict__ Fr) {
  extern __shared__ float2 gl_sm[];
  float2* x = gl_sm;          // [n]
  float2* tw = gl_sm + n;     // [n/2]
  const int t = blockIdx.x, F = n / 2 + 1;
  for (int k = threadIdx.x; k < n / 2; k += GL_NT) tw[k] = tw_g[k];
  for (int k = threadIdx.x; k < F; k += GL_NT) {
    const float s = S[(long)t * F + k];
    float2 v = ang ? ang[(long)t * F + k] : make_float2(1.f, 0.f);
    v.x *= s;
    v.y *= s;
    if (k == 0 || k == n / 2) v.y = 0.f;  // irfft ignores the imaginary part of DC / Nyquist
    x[gl_brev(k, lg)] = v;
    if (k > 0 && k < n / 2) x[gl_brev(n - k, lg)] = make_float2(v.x, -v.y);
  }
  __syncthreads();
  gl_fft(x, tw, n, lg, true);
  const float inv_n = 1.f / (float)n;
  for (int i = threadIdx.x; i < win; i += GL_NT) Fr[(long)t * win + i] = x[i].x * inv_n * gl_hann(win_g, i);
}

// One frame: samples y[t·hop + i], i < win, gathered from every frame of Fr that covers them
// (overlap-add), windowed, zero-padded to n, rfft, unit phasor est / max(1e-8, |est|) -> ang.
__global__ __launch_bounds__(GL_NT) void k_gl_stft(const float* __restrict__ Fr, int T, int hop, int win,
                                                   const float2* __restrict__ tw_g, const float* __restrict__ win_g,
                                                   int n, int lg, float2* __restrict__ ang) {
  extern __shared__ float2 gl_sm[];
  float2* x = gl_sm;
  float2* tw = gl_sm + n;
  const int t = blockIdx.x, F = n / 2 + 1;
  for (int k = threadIdx.x; k < n / 2; k += GL_NT) tw[k] = tw_g[k];
  for (int i = threadIdx.x; i < n; i += GL_NT) {
    float v = 0.f;
    if (i < win) {
      const long s = (long)t * hop + i;           // absolute sample index
      const int t1 = (int)min((long)T - 1, s / hop);
      for (int tt = t1; tt >= 0 && (long)tt * hop + win > s; --tt) v += Fr[(long)tt * win + (s - (long)tt * hop)];
      v *= gl_hann(win_g, i);
    }
    x[gl_brev(i, lg)] = make_float2(v, 0.f);
  }
  __syncthreads();
  gl_fft(x, tw, n, lg, false);
  for (int k = threadIdx.x; k < F; k += GL_NT) {
    const float2 e = x[k];
    const float m = fmaxf(1e-8f, sqrtf(e.x * e.x + e.y * e.y));
    ang[(long)t * F + k] = make_float2(e.x / m, e.y / m);
  }
}

__global__ void k_gl_ola(const float* __restrict__ Fr, int T, int hop, int win, float* __restrict__ y) {
  const long L = (long)(T - 1) * hop + win;
  for (long s = blockIdx.x * (long)blockDim.x + threadIdx.x; s < L; s += (long)gridDim.x * blockDim.x) {
    const int t1 = (int)min((long)T - 1, s / hop);
    float v = 0.f;
    for (int tt = t1; tt >= 0 && (long)tt * hop + win > s; --tt) v += Fr[(long)tt * win + (s - (long)tt * hop)];
    y[s] = v;
  }
}

}  // namespace tt2

struct tt2_gl_ctx {
  tt2_gl_config cfg;
  int dev = 0;
  int lg = 0;
  hipStream_t stream = nullptr;
  tt2::DevBuf tw, win, ib, in, amp, spec, ang, fr, wav;
};

namespace tt2 {

static GlNorm gl_norm(const tt2_gl_config& c) {
  GlNorm n;
  n.max_abs = c.max_abs_value;
  n.min_db = c.min_level_db;
  n.ref_db = c.ref_level_db;
  n.inv_mp = 1.f / c.magnitude_power;
  n.symmetric = c.symmetric_mels;
  n.clip = c.allow_clipping_in_normalization;
  return n;
}

// input [T][M or F] (device) -> waveform [(T-1)·hop + win] (device), on stream s
static void gl_run(tt2_gl_ctx* c, const float* in_d, int T, int is_mel, int iters, float* wav_d, hipStream_t s) {
  const auto& g = c->cfg;
  const int n = g.n_fft, F = n / 2 + 1, M = is_mel ? g.num_mels : 0, C = is_mel ? g.num_mels : F;
  TT2_CHECK(T >= 1, TT2_ERR_SHAPE_MISMATCH, "griffin-lim: no frames");
  TT2_CHECK(!is_mel || c->ib.p, TT2_ERR_NOT_LOADED, "griffin-lim: inverse mel basis not set");
  c->amp.alloc(sizeof(float) * T * C);
  c->spec.alloc(sizeof(float) * T * F);
  c->ang.alloc(sizeof(float2) * T * F);
  c->fr.alloc(sizeof(float) * T * g.win_size);
  const long nc = (long)T * C;
  hipLaunchKernelGGL(k_gl_amp, dim3((unsigned)std::min<long>((nc + 255) / 256, 4096)), dim3(256), 0, s, in_d, nc,
                     gl_norm(g), c->amp.as<float>());
  TT2_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_gl_spec, dim3(cdiv(F, GL_NT), T), dim3(GL_NT), 0, s, c->amp.as<float>(), c->ib.as<float>(), M,
                     F, g.power, c->spec.as<float>());
  TT2_HIP(hipGetLastError());
  const size_t shm = sizeof(float2) * (size_t)(n + n / 2);
  const float2* tw = c->tw.as<float2>();
  const float* wn = c->win.as<float>();
  hipLaunchKernelGGL(k_gl_istft, dim3(T), dim3(GL_NT), shm, s, c->spec.as<float>(), nullptr, tw, wn, n, c->lg,
                     g.win_size, c->fr.as<float>());
  TT2_HIP(hipGetLastError());
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(k_gl_stft, dim3(T), dim3(GL_NT), shm, s, c->fr.as<float>(), T, g.hop_size, g.win_size, tw, wn,
                       n, c->lg, c->ang.as<float2>());
    TT2_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_gl_istft, dim3(T), dim3(GL_NT), shm, s, c->spec.as<float>(), c->ang.as<float2>(), tw, wn, n,
                       c->lg, g.win_size, c->fr.as<float>());
    TT2_HIP(hipGetLastError());
  }
  const long L = (long)(T - 1) * g.hop_size + g.win_size;
  hipLaunchKernelGGL(k_gl_ola, dim3((unsigned)std::min<long>((L + 255) / 256, 4096)), dim3(256), 0, s,
                     c->fr.as<float>(), T, g.hop_size, g.win_size, wav_d);
  TT2_HIP(hipGetLastError());
}

}  // namespace tt2

using namespace tt2;

extern "C" {

void tt2_gl_default_config(tt2_gl_config* c) {
  c->n_fft = 2048; c->hop_size = 275; c->win_size = 1100; c->num_mels = 80;
  c->magnitude_power = 2.f; c->power = 1.5f; c->ref_level_db = 20.f; c->min_level_db = -100.f;
  c->max_abs_value = 4.f; c->symmetric_mels = 1; c->allow_clipping_in_normalization = 1;
  c->griffin_lim_iters = 60;
}

tt2_status tt2_gl_create(const tt2_gl_config* cfg, int hip_device, tt2_gl_ctx** out) {
  return guard([&] {
    TT2_CHECK(cfg && out, TT2_ERR_INVALID_ARG, "tt2_gl_create: null argument");
    *out = nullptr;
    const int n = cfg->n_fft;
    int lg = 0;
    while ((1 << lg) < n) ++lg;
    TT2_CHECK(n >= 16 && n <= GL_MAX_FFT && (1 << lg) == n, TT2_ERR_INVALID_ARG,
              "n_fft must be a power of two in [16, 4096]");
    TT2_CHECK(cfg->win_size >= 1 && cfg->win_size <= n, TT2_ERR_INVALID_ARG, "win_size must be in [1, n_fft]");
    TT2_CHECK(cfg->hop_size >= 1 && cfg->hop_size <= cfg->win_size, TT2_ERR_INVALID_ARG, "hop_size must be in [1, win_size]");
    TT2_CHECK(cfg->num_mels >= 1 && cfg->num_mels <= 256, TT2_ERR_INVALID_ARG, "num_mels must be in [1, 256]");
    TT2_CHECK(cfg->magnitude_power > 0.f && cfg->griffin_lim_iters >= 0, TT2_ERR_INVALID_ARG, "bad power / iters");
    int ndev = 0;
    TT2_HIP(hipGetDeviceCount(&ndev));
    TT2_CHECK(hip_device >= 0 && hip_device < ndev, TT2_ERR_INVALID_ARG, "tt2_gl_create: bad device index");
    auto c = std::make_unique<tt2_gl_ctx>();
    c->cfg = *cfg;
    c->dev = hip_device;
    c->lg = lg;
    TT2_HIP(hipSetDevice(hip_device));
    TT2_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    std::vector<float2> tw(n / 2);
    for (int k = 0; k < n / 2; ++k) {
      const double a = -2.0 * M_PI * k / n;
      tw[k] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    c->tw.alloc(sizeof(float2) * tw.size());
    TT2_HIP(hipMemcpy(c->tw.p, tw.data(), sizeof(float2) * tw.size(), hipMemcpyHostToDevice));
    std::vector<float> w(cfg->win_size);
    for (int i = 0; i < cfg->win_size; ++i) w[i] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * i / cfg->win_size));
    c->win.alloc(sizeof(float) * w.size());
    TT2_HIP(hipMemcpy(c->win.p, w.data(), sizeof(float) * w.size(), hipMemcpyHostToDevice));
    *out = c.release();
  });
}

void tt2_gl_destroy(tt2_gl_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

tt2_status tt2_gl_set_inv_mel_basis(tt2_gl_ctx* c, const float* inv_basis) {
  return guard([&] {
    TT2_CHECK(c && inv_basis, TT2_ERR_INVALID_ARG, "tt2_gl_set_inv_mel_basis: null argument");
    TT2_HIP(hipSetDevice(c->dev));
    const size_t bytes = sizeof(float) * (size_t)(c->cfg.n_fft / 2 + 1) * c->cfg.num_mels;
    c->ib.alloc(bytes);
    TT2_HIP(hipMemcpy(c->ib.p, inv_basis, bytes, hipMemcpyHostToDevice));
  });
}

tt2_status tt2_gl_synthesize(tt2_gl_ctx* c, const float* spec, int T, int is_mel, int iters, float* wav_out) {
  return guard([&] {
    TT2_CHECK(c && spec && wav_out, TT2_ERR_INVALID_ARG, "tt2_gl_synthesize: null argument");
    TT2_CHECK(T >= 1, TT2_ERR_SHAPE_MISMATCH, "tt2_gl_synthesize: T must be >= 1");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    const int C = is_mel ? c->cfg.num_mels : c->cfg.n_fft / 2 + 1;
    const long L = (long)(T - 1) * c->cfg.hop_size + c->cfg.win_size;
    c->in.alloc(sizeof(float) * T * C);
    c->wav.alloc(sizeof(float) * L);
    TT2_HIP(hipMemcpyAsync(c->in.p, spec, sizeof(float) * T * C, hipMemcpyHostToDevice, s));
    gl_run(c, c->in.as<float>(), T, is_mel, iters < 0 ? c->cfg.griffin_lim_iters : iters, c->wav.as<float>(), s);
    TT2_HIP(hipMemcpyAsync(wav_out, c->wav.p, sizeof(float) * L, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
  });
}

tt2_status tt2_gl_synthesize_dev(tt2_gl_ctx* c, const float* spec_d, int T, int is_mel, int iters, float* wav_d,
                                 void* stream) {
  return guard([&] {
    TT2_CHECK(c && spec_d && wav_d, TT2_ERR_INVALID_ARG, "tt2_gl_synthesize_dev: null argument");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    gl_run(c, spec_d, T, is_mel, iters < 0 ? c->cfg.griffin_lim_iters : iters, wav_d, s);
  });
}

}  // extern "C"
