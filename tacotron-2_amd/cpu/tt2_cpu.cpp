// libtt2_cpu.so — the synthesis subset of the libtt2 C ABI (include/tt2.h) on host CPU cores:
// fp32, OpenMP, register-blocked GEMM.  Same entry points, argument meaning and error behaviour
// as the HIP library, so a caller binds either file; this one is the timed CPU baseline of
// bench.py (a C++ restatement of the reference path, not TensorFlow) and a second, independent
// implementation the CPU test suite checks against the numpy oracle.
//
// Exported: tt2_last_error, tt2_version, tt2_default_config, tt2_create, tt2_destroy,
// tt2_load_tensor, tt2_finalize_weights, tt2_encode, tt2_decode, tt2_decoder_step, tt2_postnet,
// tt2_prenet_keep_bits; tt2_wn_default_config, tt2_wn_create, tt2_wn_destroy, tt2_wn_load_tensor,
// tt2_wn_finalize, tt2_wn_generate, tt2_wn_noise, tt2_mol_sample.  The *_dev / training /
// Griffin-Lim / profiling entry points and the Tacotron_emt_attn variant are GPU-only.
//
// Reference (code/): tacotron/models/{tacotron.py:215-381, modules.py, attention.py:10-227,
// Architecture_wrappers.py:197-267, helpers.py:6-133, multihead_attention.py:35-132},
// wavenet_vocoder/models/{wavenet.py:724-911, modules.py:270-297, 497-520, 524-770, mixture.py:76-107,
// gaussian.py:39-52}.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include <omp.h>

#include "../../include/tt2.h"
#include "../csrc/rng.h"

namespace {

thread_local std::string g_err;

struct Error : std::runtime_error {
  int status;
  Error(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};
#define CK(cond, st, msg)                   \
  do {                                      \
    if (!(cond)) throw Error((st), (msg));  \
  } while (0)

template <class F>
tt2_status guard(F&& f) {
  try {
    f();
    return TT2_OK;
  } catch (const Error& e) {
    g_err = e.what();
    return e.status;
  } catch (const std::exception& e) {
    g_err = e.what();
    return TT2_ERR_INVALID_ARG;
  }
}

struct Tensor {
  std::vector<int64_t> shape;
  std::vector<float> v;
};
using WeightMap = std::map<std::string, Tensor>;

void put(WeightMap& wm, const char* name, const float* host, const int64_t* shape, int ndim) {
  CK(name && (host || ndim == 0) && ndim >= 0 && ndim <= 8, TT2_ERR_INVALID_ARG, "load_tensor: bad argument");
  Tensor t;
  size_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    CK(shape[i] >= 0, TT2_ERR_INVALID_ARG, "load_tensor: negative dimension");
    t.shape.push_back(shape[i]);
    n *= (size_t)shape[i];
  }
  t.v.assign(host, host + n);
  wm[name] = std::move(t);
}

const std::vector<float>& need(const WeightMap& wm, const std::string& name, std::vector<int64_t> shape) {
  auto it = wm.find(name);
  CK(it != wm.end(), TT2_ERR_NOT_LOADED, "missing variable " + name);
  auto squeeze = [](const std::vector<int64_t>& v) {  // scalars may come as () or (1,)
    std::vector<int64_t> r;
    for (auto d : v)
      if (d != 1) r.push_back(d);
    return r;
  };
  CK(squeeze(it->second.shape) == squeeze(shape), TT2_ERR_SHAPE_MISMATCH, "shape mismatch for " + name);
  return it->second.v;
}

// ---- dense algebra --------------------------------------------------------------------------------

// y[m][n] (+)= Σ_k x[m·ldx + k]·W[k·N + n] (+ bias[n]).  Rows of x may overlap (ldx < K: the
// implicit im2col of a 'same' conv over a time-padded input).  W is repacked once into 16-column
// strips [N/16][K][16] (zero-padded), so a strip streams contiguously; register tiles of R rows x
// 16 columns (two 8-wide vectors per row) accumulate over all of K; OpenMP over (strip, row chunk).
typedef float v8 __attribute__((vector_size(32)));

std::map<std::tuple<const float*, int, int>, std::vector<float>> g_pack;  // by (weights, K, N)

// packed strips of a weight matrix; the cache is dropped whenever any weights are (re)loaded or a
// context is destroyed, so a key never outlives the storage it names
const float* packed(const float* W, int K, int N) {
  const auto key = std::make_tuple(W, K, N);
  auto it = g_pack.find(key);
  if (it != g_pack.end()) return it->second.data();
  const int NS = (N + 15) / 16;
  std::vector<float> p((size_t)NS * K * 16, 0.f);
  for (int s = 0; s < NS; ++s)
    for (int k = 0; k < K; ++k)
      for (int c = 0; c < 16 && 16 * s + c < N; ++c) p[((size_t)s * K + k) * 16 + c] = W[(size_t)k * N + 16 * s + c];
  return g_pack.emplace(key, std::move(p)).first->second.data();
}

template <int R>
inline void tile(const float* __restrict x, long ldx, int K, const float* __restrict Ws, int ncols,
                 float* __restrict y, long ldy, bool accum) {
  v8 acc[R][2];
  for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = (v8){0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < K; ++k) {
    v8 w0, w1;
    std::memcpy(&w0, Ws + (size_t)k * 16, 32);
    std::memcpy(&w1, Ws + (size_t)k * 16 + 8, 32);
#pragma GCC unroll 8
    for (int r = 0; r < R; ++r) {
      const float xv = x[r * ldx + k];
      acc[r][0] += xv * w0;
      acc[r][1] += xv * w1;
    }
  }
  for (int r = 0; r < R; ++r) {
    float o[16];
    std::memcpy(o, &acc[r][0], 32);
    std::memcpy(o + 8, &acc[r][1], 32);
    for (int c = 0; c < ncols; ++c) y[r * ldy + c] = accum ? y[r * ldy + c] + o[c] : o[c];
  }
}

void gemm(const float* x, int M, int K, long ldx, const float* W, int N, const float* bias, float* y, long ldy,
          bool accum = false) {
  const float* Wp = packed(W, K, N);
  const int NS = (N + 15) / 16, MB = 6;
  // row chunks: enough (strip, chunk) tasks for the thread pool, chunks a multiple of MB rows
  const int nmc0 = std::max(1, std::min((M + MB - 1) / MB, (4 * omp_get_max_threads() + NS - 1) / NS));
  const int mchunk = ((M + nmc0 - 1) / nmc0 + MB - 1) / MB * MB;
  const int nmc = (M + mchunk - 1) / mchunk;
  const long work = (long)M * N * K;
#pragma omp parallel for collapse(2) schedule(dynamic) if (work > (1L << 18))
  for (int s = 0; s < NS; ++s)
    for (int mc = 0; mc < nmc; ++mc) {
      const int m_end = std::min(M, (mc + 1) * mchunk), n0 = 16 * s, nc = std::min(16, N - n0);
      const float* Ws = Wp + (size_t)s * K * 16;
      int m = mc * mchunk;
      for (; m + MB <= m_end; m += MB) tile<MB>(x + (long)m * ldx, ldx, K, Ws, nc, y + (long)m * ldy + n0, ldy, accum);
      for (; m < m_end; ++m) tile<1>(x + (long)m * ldx, ldx, K, Ws, nc, y + (long)m * ldy + n0, ldy, accum);
      if (bias)
        for (int r = mc * mchunk; r < m_end; ++r)
          for (int c = 0; c < nc; ++c) y[(long)r * ldy + n0 + c] += bias[n0 + c];
    }
}

inline float sigm(float x) { return 1.f / (1.f + std::exp(-x)); }

// tf.layers.batch_normalization(training=False) as TF computes it: x·inv + (beta − mean·inv)
struct BN {
  std::vector<float> inv, sh;
};
BN bn_consts(const WeightMap& wm, const std::string& sc, int C) {
  const auto& g = need(wm, sc + "batch_normalization/gamma", {C});
  const auto& be = need(wm, sc + "batch_normalization/beta", {C});
  const auto& mu = need(wm, sc + "batch_normalization/moving_mean", {C});
  const auto& var = need(wm, sc + "batch_normalization/moving_variance", {C});
  BN r;
  r.inv.resize(C);
  r.sh.resize(C);
  for (int c = 0; c < C; ++c) {
    r.inv[c] = g[c] / std::sqrt(var[c] + 1e-3f);
    r.sh[c] = be[c] - mu[c] * r.inv[c];
  }
  return r;
}

// conv1d 'same' stride 1 (modules.py:485-497 conv1d with bnorm='after'): y = BN(act(conv + b)).
// x [B][T][C] -> y [B][T][O]; the time-padded copy makes every output row's taps one contiguous
// k·C slice (implicit im2col, rows overlapping by C).  act: 0 none, 1 relu, 2 tanh.
void conv1d_bn(const float* x, int B, int T, int C, const std::vector<float>& k, int kw, int O,
               const std::vector<float>& b, const BN& bn, int act, float* y) {
  const int pl = (kw - 1) / 2, Tp = T + kw - 1;
  std::vector<float> xp((size_t)B * Tp * C, 0.f);
  for (int bb = 0; bb < B; ++bb)
    std::memcpy(&xp[((size_t)bb * Tp + pl) * C], x + (size_t)bb * T * C, sizeof(float) * T * C);
  for (int bb = 0; bb < B; ++bb)
    gemm(&xp[(size_t)bb * Tp * C], T, kw * C, C, k.data(), O, b.data(), y + (size_t)bb * T * O, O);
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)B * T; ++i) {
    float* r = y + i * O;
    for (int o = 0; o < O; ++o) {
      float v = r[o];
      if (act == 1) v = std::max(v, 0.f);
      else if (act == 2) v = std::tanh(v);
      r[o] = v * bn.inv[o] + bn.sh[o];
    }
  }
}

}  // namespace

// =====================================================================================================
// Tacotron-2
// =====================================================================================================
struct tt2_ctx {
  tt2_config cfg;
  WeightMap wm;
  bool finalized = false;
  int nm, E, Cenc, U, A, F, KL, P, H, PC, Dm, SW, nref, nmel, style_mode;
  // encoded batch
  int B = 0, T_in = 0;
  bool encoded = false, decoded = false;
  std::vector<int> lens;
  std::vector<float> values, keys, style;  // [B][T][Dm], [B][T][A], [B][SW]
  // last decode
  int n_steps = 0, max_iters_last = 0;
  std::vector<float> frames;               // [B][max_iters * r][nm]
};

namespace {

const char* TP = "Tacotron_model/inference/";

const std::vector<float>& W(const tt2_ctx* c, const std::string& n, std::vector<int64_t> s) {
  return need(c->wm, TP + n, std::move(s));
}

// tf.nn.bidirectional_dynamic_rnn over Zoneout-LSTM cells with sequence_length (modules.py:313-323):
// past a row's length the output is 0 and the state is carried; bw runs on the length-reversed
// input and is reversed back.  x [B][T][C] -> out [B][T][2U].
void bilstm(tt2_ctx* c, const float* x, int B, int T, int C, float* out) {
  const int U = c->U;
  const float z = c->cfg.zoneout, omz = (float)(1.0 - (double)c->cfg.zoneout);
  std::fill(out, out + (size_t)B * T * 2 * U, 0.f);
  for (int d = 0; d < 2; ++d) {
    const std::string s = std::string("encoder_LSTM/bidirectional_rnn/") + (d ? "bw" : "fw") + "/lstm_cell/";
    const auto& k = W(c, s + "kernel", {C + U, 4 * U});
    const auto& b = W(c, s + "bias", {4 * U});
    std::vector<float> xp((size_t)B * T * 4 * U);
    gemm(x, B * T, C, C, k.data(), 4 * U, b.data(), xp.data(), 4 * U);
    std::vector<float> h((size_t)B * U, 0.f), cc((size_t)B * U, 0.f), zr((size_t)B * 4 * U);
    int Tmax = 0;
    for (int bb = 0; bb < B; ++bb) Tmax = std::max(Tmax, c->lens[bb]);
    for (int t = 0; t < Tmax; ++t) {
      gemm(h.data(), B, U, U, k.data() + (size_t)C * 4 * U, 4 * U, nullptr, zr.data(), 4 * U);
      for (int bb = 0; bb < B; ++bb) {
        const int L = c->lens[bb];
        if (t >= L) continue;
        const int pos = d ? L - 1 - t : t;
        const float* g0 = &xp[((size_t)bb * T + pos) * 4 * U];
        const float* g1 = &zr[(size_t)bb * 4 * U];
        for (int u = 0; u < U; ++u) {
          const float zi = g0[u] + g1[u], zj = g0[U + u] + g1[U + u], zf = g0[2 * U + u] + g1[2 * U + u],
                      zo = g0[3 * U + u] + g1[3 * U + u];
          const float cp = cc[(size_t)bb * U + u], hp = h[(size_t)bb * U + u];
          const float cn = sigm(zf + 1.f) * cp + sigm(zi) * std::tanh(zj);
          const float hn = sigm(zo) * std::tanh(cn);
          out[((size_t)bb * T + pos) * 2 * U + d * U + u] = hn;
          cc[(size_t)bb * U + u] = omz * cn + z * cp;
          h[(size_t)bb * U + u] = omz * hn + z * hp;
        }
      }
    }
  }
}

// ReferenceEncoder CNN stack (modules.py:20-33; conv2d() :499-511 = conv, BN, ReLU) or, adain,
// ReferenceEncoderAdaIn's (modules.py:75-87: conv + ReLU, no BN, strides (2,2),(2,2),(1,1)x4):
// mel [B][TR][nm] -> NHWC [B][H][W][C]
std::vector<float> conv_stack(tt2_ctx* c, const std::string& s, const float* mel, int B, int TR, bool adain, int& H,
                              int& Wd, int& C, const char* layer = "conv2d") {
  const auto& cfg = c->cfg;
  std::vector<float> x(mel, mel + (size_t)B * TR * c->nm), y;
  H = TR; Wd = c->nm; C = 1;
  for (int i = 0; i < 6; ++i) {
    const std::string s2 = s + "conv2d_" + std::to_string(i) + "/";
    const int f = cfg.reference_filters[i], st = adain && i >= 2 ? 1 : 2;
    const auto& k = W(c, s2 + layer + "/kernel", {3, 3, C, f});
    const auto& bi = W(c, s2 + layer + "/bias", {f});
    BN bn;
    if (!adain) bn = bn_consts(c->wm, TP + s2, f);
    const int Ho = (H + st - 1) / st, Wo = (Wd + st - 1) / st;
    const int pt = std::max((Ho - 1) * st + 3 - H, 0) / 2, pl = std::max((Wo - 1) * st + 3 - Wd, 0) / 2;
    const long rows = (long)B * Ho * Wo;
    std::vector<float> col(rows * 9 * C, 0.f);
#pragma omp parallel for schedule(static)
    for (long r = 0; r < rows; ++r) {
      const int bb = (int)(r / ((long)Ho * Wo)), ho = (int)(r / Wo % Ho), wo = (int)(r % Wo);
      for (int ki = 0; ki < 3; ++ki)
        for (int kj = 0; kj < 3; ++kj) {
          const int hi = ho * st + ki - pt, wi = wo * st + kj - pl;
          if (hi < 0 || hi >= H || wi < 0 || wi >= Wd) continue;
          std::memcpy(&col[(r * 9 + ki * 3 + kj) * C], &x[(((size_t)bb * H + hi) * Wd + wi) * C], sizeof(float) * C);
        }
    }
    y.assign(rows * f, 0.f);
    gemm(col.data(), (int)rows, 9 * C, 9 * C, k.data(), f, bi.data(), y.data(), f);
    for (long i2 = 0; i2 < rows; ++i2)
      for (int o = 0; o < f; ++o) {
        const float v = adain ? y[i2 * f + o] : y[i2 * f + o] * bn.inv[o] + bn.sh[o];
        y[i2 * f + o] = std::max(v, 0.f);
      }
    x.swap(y);
    H = Ho; Wd = Wo; C = f;
  }
  return x;
}

// GRU over every frame, last output -> dense(128, tanh) (modules.py:57-64): x [B][H][gin] -> ref
std::vector<float> gru_dense(tt2_ctx* c, const std::string& s, const float* x, int B, int H, int gin) {
  const int D = c->cfg.reference_depth;
  const auto& kg = W(c, s + "rnn/gru_cell/gates/kernel", {gin + D, 2 * D});
  const auto& bg = W(c, s + "rnn/gru_cell/gates/bias", {2 * D});
  const auto& kc = W(c, s + "rnn/gru_cell/candidate/kernel", {gin + D, D});
  const auto& bc = W(c, s + "rnn/gru_cell/candidate/bias", {D});
  std::vector<float> h((size_t)B * D, 0.f), g((size_t)B * 2 * D), cd((size_t)B * D), rh((size_t)B * D);
  std::vector<float> xg((size_t)B * H * 2 * D), xc((size_t)B * H * D);
  gemm(x, B * H, gin, gin, kg.data(), 2 * D, bg.data(), xg.data(), 2 * D);
  gemm(x, B * H, gin, gin, kc.data(), D, bc.data(), xc.data(), D);
  for (int t = 0; t < H; ++t) {
    gemm(h.data(), B, D, D, kg.data() + (size_t)gin * 2 * D, 2 * D, nullptr, g.data(), 2 * D);
    for (int bb = 0; bb < B; ++bb)
      for (int j = 0; j < 2 * D; ++j) g[(size_t)bb * 2 * D + j] = sigm(g[(size_t)bb * 2 * D + j] + xg[((size_t)bb * H + t) * 2 * D + j]);
    for (int bb = 0; bb < B; ++bb)
      for (int i = 0; i < D; ++i) rh[(size_t)bb * D + i] = g[(size_t)bb * 2 * D + i] * h[(size_t)bb * D + i];
    gemm(rh.data(), B, D, D, kc.data() + (size_t)gin * D, D, nullptr, cd.data(), D);
    for (int bb = 0; bb < B; ++bb)
      for (int i = 0; i < D; ++i) {
        const float cand = std::tanh(cd[(size_t)bb * D + i] + xc[((size_t)bb * H + t) * D + i]);
        const float u = g[(size_t)bb * 2 * D + D + i];
        h[(size_t)bb * D + i] = u * h[(size_t)bb * D + i] + (1.f - u) * cand;
      }
  }
  std::vector<float> ref((size_t)B * 128);
  gemm(h.data(), B, D, D, W(c, s + "dense/kernel", {D, 128}).data(), 128, W(c, s + "dense/bias", {128}).data(),
       ref.data(), 128);
  for (auto& v : ref) v = std::tanh(v);
  return ref;
}

// GST MultiheadAttention (multihead_attention.py:35-132, tacotron.py:276-282): values tanh(tokens);
// q = ref·Wq + bq; k = values·Wk + bk; per head normed_v·tanh(k + q + b), softmax over tokens,
// context = weights·values (every head sees all tokd channels), heads concatenated into style
void gst(tt2_ctx* c, const char* tag, const std::vector<float>& ref, int B, float* style, int off) {
  const auto& cfg = c->cfg;
  const int ntok = cfg.num_gst, heads = cfg.num_heads, tokd = cfg.style_embed_depth / heads, Aa = cfg.style_att_dim;
  const int dh = Aa / heads;
  const std::string mh = std::string("Multihead-attention-") + tag + "/";
  std::vector<float> vals(W(c, std::string("style_tokens_") + tag, {ntok, tokd}));
  for (auto& v : vals) v = std::tanh(v);
  std::vector<float> q((size_t)B * Aa), kk((size_t)ntok * Aa);
  gemm(ref.data(), B, 128, 128, W(c, mh + "conv1d/kernel", {1, 128, Aa}).data(), Aa,
       W(c, mh + "conv1d/bias", {Aa}).data(), q.data(), Aa);
  gemm(vals.data(), ntok, tokd, tokd, W(c, mh + "conv1d_1/kernel", {1, tokd, Aa}).data(), Aa,
       W(c, mh + "conv1d_1/bias", {Aa}).data(), kk.data(), Aa);
  const auto& av = W(c, mh + "attention_v", {dh});
  const float ag = W(c, mh + "attention_g", {})[0];
  const auto& ab = W(c, mh + "attention_b", {dh});
  float ss = 0.f;
  for (float v : av) ss += v * v;
  const float r = 1.f / std::sqrt(ss);
  for (int bb = 0; bb < B; ++bb)
    for (int hh = 0; hh < heads; ++hh) {
      std::vector<float> sc(ntok);
      float mx = -INFINITY;
      for (int tk = 0; tk < ntok; ++tk) {
        float a = 0.f;
        for (int d = 0; d < dh; ++d)
          a += (ag * av[d] * r) * std::tanh(kk[(size_t)tk * Aa + hh * dh + d] + q[(size_t)bb * Aa + hh * dh + d] + ab[d]);
        sc[tk] = a;
        mx = std::max(mx, a);
      }
      float sum = 0.f;
      for (auto& v : sc) sum += (v = std::exp(v - mx));
      for (int d = 0; d < tokd; ++d) {
        float acc = 0.f;
        for (int tk = 0; tk < ntok; ++tk) acc += (sc[tk] / sum) * vals[(size_t)tk * tokd + d];
        style[(size_t)bb * c->SW + off + hh * tokd + d] = acc;
      }
    }
}

// ReferenceEncoderAdaIn (modules.py:89-107): per (row, channel) moments over (time, freq) of both
// maps; spk = 0.9·spk + 0.1·batch_normalization(spk, m_s, v_s, offset=m_e, scale=v_e, 1e-9)
void adain_mix(std::vector<float>& spk, const std::vector<float>& emt, int B, int HWs, int HWe, int C) {
  auto moments = [&](const std::vector<float>& x, int HW, std::vector<float>& m, std::vector<float>& v) {
    m.assign((size_t)B * C, 0.f);
    v.assign((size_t)B * C, 0.f);
    for (int b = 0; b < B; ++b)
      for (int ch = 0; ch < C; ++ch) {
        double s1 = 0.0;
        for (int i = 0; i < HW; ++i) s1 += x[((size_t)b * HW + i) * C + ch];
        const float mean = (float)(s1 / HW);
        double s2 = 0.0;
        for (int i = 0; i < HW; ++i) {
          const float d = x[((size_t)b * HW + i) * C + ch] - mean;
          s2 += (double)d * d;
        }
        m[(size_t)b * C + ch] = mean;
        v[(size_t)b * C + ch] = (float)(s2 / HW);
      }
  };
  std::vector<float> ms, vs, me, ve;
  moments(spk, HWs, ms, vs);
  moments(emt, HWe, me, ve);
  for (int b = 0; b < B; ++b)
    for (int i = 0; i < HWs; ++i)
      for (int ch = 0; ch < C; ++ch) {
        const size_t k = (size_t)b * C + ch;
        const float inv = (1.f / std::sqrt(vs[k] + 1e-9f)) * ve[k];
        float& x = spk[((size_t)b * HWs + i) * C + ch];
        x = x * 0.9f + (x * inv + (me[k] - ms[k] * inv)) * 0.1f;
      }
}

void encode(tt2_ctx* c, const int* ids, const int* lengths, int B, int T, const float* ref[2], const int TR[2]) {
  const auto& cfg = c->cfg;
  CK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_finalize_weights not called");
  CK(B >= 1 && B <= cfg.max_batch, TT2_ERR_SHAPE_MISMATCH, "batch exceeds capacity");
  CK(T >= 1 && T <= cfg.max_T_in, TT2_ERR_SHAPE_MISMATCH, "T_in exceeds capacity");
  c->lens.assign(lengths, lengths + B);
  for (int b = 0; b < B; ++b)
    CK(c->lens[b] >= 1 && c->lens[b] <= T, TT2_ERR_INVALID_ARG, "input_lengths must be in [1, T_in]");
  // embedding + 3 x conv(relu) + BN (tacotron.py:215-231, modules.py:274-280)
  const auto& emb = W(c, "inputs_embedding", {cfg.n_symbols, c->E});
  std::vector<float> x((size_t)B * T * c->E);
  for (int i = 0; i < B * T; ++i) {
    const int id = ids[i];
    CK(id >= 0 && id < cfg.n_symbols, TT2_ERR_INVALID_ARG, "symbol id out of range");
    std::memcpy(&x[(size_t)i * c->E], &emb[(size_t)id * c->E], sizeof(float) * c->E);
  }
  int cin = c->E;
  std::vector<float> y;
  for (int i = 1; i <= cfg.enc_conv_num_layers; ++i) {
    const std::string s = "encoder_convolutions/conv_layer_" + std::to_string(i) + "_encoder_convolutions/";
    y.assign((size_t)B * T * c->Cenc, 0.f);
    conv1d_bn(x.data(), B, T, cin, W(c, s + "conv1d/kernel", {cfg.enc_conv_kernel_size, cin, c->Cenc}),
              cfg.enc_conv_kernel_size, c->Cenc, W(c, s + "conv1d/bias", {c->Cenc}), bn_consts(c->wm, TP + s, c->Cenc),
              1, y.data());
    x.swap(y);
    cin = c->Cenc;
  }
  std::vector<float> enc((size_t)B * T * 2 * c->U);
  bilstm(c, x.data(), B, T, cin, enc.data());
  // reference encoders + style (tacotron.py:236-308): GST, the embeddings themselves, or AdaIN
  c->style.assign((size_t)B * std::max(c->SW, 1), 0.f);
  const char* tags[2] = {"emt", "spk"};
  for (int r = 0; r < c->nmel; ++r)
    CK(ref[r] && TR[r] >= 1 && TR[r] <= cfg.max_T_ref, TT2_ERR_SHAPE_MISMATCH, "T_ref exceeds capacity");
  int H, Wd, C;
  if (c->style_mode == 2) {
    int He, We, Ce;
    // the emotion stack's convs are conv2d_i/conv2d_1/* (weights.py _adain_refnet_specs)
    const std::vector<float> xe = conv_stack(c, "refnet/", ref[0], B, TR[0], true, He, We, Ce, "conv2d_1");
    std::vector<float> xs = conv_stack(c, "refnet/", ref[1], B, TR[1], true, H, Wd, C);
    adain_mix(xs, xe, B, H * Wd, He * We, C);
    const auto r = gru_dense(c, "refnet/", xs.data(), B, H, Wd * C);
    for (int b = 0; b < B; ++b) std::memcpy(&c->style[(size_t)b * c->SW], &r[(size_t)b * 128], sizeof(float) * 128);
  } else {
    for (int r = 0; r < c->nref; ++r) {
      const std::string sc = std::string("refnet_") + tags[r] + "/";
      const std::vector<float> x = conv_stack(c, sc, ref[r], B, TR[r], false, H, Wd, C);
      const auto e = gru_dense(c, sc, x.data(), B, H, Wd * C);
      if (c->style_mode == 0) {
        gst(c, tags[r], e, B, c->style.data(), r * cfg.style_embed_depth);
      } else {
        for (int b = 0; b < B; ++b)
          std::memcpy(&c->style[(size_t)b * c->SW + r * 128], &e[(size_t)b * 128], sizeof(float) * 128);
      }
    }
  }
  // values = [enc | tiled style] masked past each row's length; keys = memory_layer(values)
  const int E2 = 2 * c->U;
  c->values.assign((size_t)B * T * c->Dm, 0.f);
  for (int b = 0; b < B; ++b)
    for (int t = 0; t < c->lens[b]; ++t) {
      float* v = &c->values[((size_t)b * T + t) * c->Dm];
      std::memcpy(v, &enc[((size_t)b * T + t) * E2], sizeof(float) * E2);
      std::memcpy(v + E2, &c->style[(size_t)b * c->SW], sizeof(float) * c->SW);
    }
  c->keys.assign((size_t)B * T * c->A, 0.f);
  gemm(c->values.data(), B * T, c->Dm, c->Dm, W(c, "memory_layer/kernel", {c->Dm, c->A}).data(), c->A, nullptr,
       c->keys.data(), c->A);
  c->B = B;
  c->T_in = T;
  c->encoded = true;
  c->decoded = false;
}

// decoder state of the batch (TacotronDecoderState, Architecture_wrappers.py:158-195)
struct DecState {
  std::vector<float> h1, c1, h2, c2, ctx, cum;
  std::vector<int> max_att;
};

// One TacotronDecoderCell.__call__ (Architecture_wrappers.py:197-267), in place on st.
void dec_step(tt2_ctx* c, const float* frame_in, const uint8_t* masks, DecState& st, float* frame, float* stop,
              float* align) {
  const auto& cfg = c->cfg;
  const int B = c->B, T = c->T_in, P = c->P, H = c->H, D = c->Dm, A = c->A, nm = c->nm;
  const float z = cfg.zoneout, omz = (float)(1.0 - (double)cfg.zoneout);
  // prenet (modules.py:346-357): dropout stays on at inference
  std::vector<float> x1((size_t)B * P), x2((size_t)B * P);
  gemm(frame_in, B, nm, nm, W(c, "decoder/decoder_prenet/dense_1/kernel", {nm, P}).data(), P,
       W(c, "decoder/decoder_prenet/dense_1/bias", {P}).data(), x1.data(), P);
  for (int i = 0; i < B * P; ++i) x1[i] = (std::max(x1[i], 0.f) / 0.5f) * (float)masks[i];
  gemm(x1.data(), B, P, P, W(c, "decoder/decoder_prenet/dense_2/kernel", {P, P}).data(), P,
       W(c, "decoder/decoder_prenet/dense_2/bias", {P}).data(), x2.data(), P);
  for (int i = 0; i < B * P; ++i) x2[i] = (std::max(x2[i], 0.f) / 0.5f) * (float)masks[B * P + i];
  // two Zoneout-LSTM layers; emitted output = raw h_new, carried state = zoneout mix
  auto lstm = [&](const std::vector<float>& xin, int K, const std::string& cell, std::vector<float>& h,
                  std::vector<float>& cs, std::vector<float>& o) {
    std::vector<float> in((size_t)B * (K + H)), zz((size_t)B * 4 * H);
    for (int b = 0; b < B; ++b) {
      std::memcpy(&in[(size_t)b * (K + H)], &xin[(size_t)b * K], sizeof(float) * K);
      std::memcpy(&in[(size_t)b * (K + H) + K], &h[(size_t)b * H], sizeof(float) * H);
    }
    const std::string s = "decoder/decoder_LSTM/multi_rnn_cell/" + cell + "/lstm_cell/";
    gemm(in.data(), B, K + H, K + H, W(c, s + "kernel", {K + H, 4 * H}).data(), 4 * H,
         W(c, s + "bias", {4 * H}).data(), zz.data(), 4 * H);
    o.resize((size_t)B * H);
    for (int b = 0; b < B; ++b)
      for (int u = 0; u < H; ++u) {
        const float* g = &zz[(size_t)b * 4 * H];
        const float cp = cs[(size_t)b * H + u], hp = h[(size_t)b * H + u];
        const float cn = sigm(g[2 * H + u] + 1.f) * cp + sigm(g[u]) * std::tanh(g[H + u]);
        const float hn = sigm(g[3 * H + u]) * std::tanh(cn);
        o[(size_t)b * H + u] = hn;
        cs[(size_t)b * H + u] = omz * cn + z * cp;
        h[(size_t)b * H + u] = omz * hn + z * hp;
      }
  };
  std::vector<float> xin((size_t)B * (P + D)), o1, o2;
  for (int b = 0; b < B; ++b) {
    std::memcpy(&xin[(size_t)b * (P + D)], &x2[(size_t)b * P], sizeof(float) * P);
    std::memcpy(&xin[(size_t)b * (P + D) + P], &st.ctx[(size_t)b * D], sizeof(float) * D);
  }
  lstm(xin, P + D, "cell_0", st.h1, st.c1, o1);
  lstm(o1, H, "cell_1", st.h2, st.c2, o2);
  // LocationSensitiveAttention (attention.py:170-227)
  const std::string la = "decoder/Location_Sensitive_Attention/";
  std::vector<float> q((size_t)B * A);
  gemm(o2.data(), B, H, H, W(c, "decoder/query_layer/kernel", {H, A}).data(), A, nullptr, q.data(), A);
  const auto& wcv = W(c, la + "location_features_convolution/kernel", {c->KL, 1, c->F});
  const auto& bcv = W(c, la + "location_features_convolution/bias", {c->F});
  const auto& wl = W(c, la + "location_features_layer/kernel", {c->F, A});
  const auto& va = W(c, la + "attention_variable_projection", {A});
  const auto& ba = W(c, la + "attention_bias", {A});
  // location features f = conv1d_same(cum) + b (attention.py:193-195), loc = f·W_loc (:197) as one
  // GEMM over every (row, encoder step), energies e = Σ_k v_a·tanh(keys + q + loc + b_a) (:69)
  const int Fw = c->F, pl = (c->KL - 1) / 2;
  std::vector<float> fl((size_t)B * T * Fw), loc((size_t)B * T * A), en((size_t)B * T);
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < T; ++j)
      for (int ff = 0; ff < Fw; ++ff) {
        float s2 = bcv[ff];
        for (int tap = 0; tap < c->KL; ++tap) {
          const int src = j + tap - pl;
          if (src >= 0 && src < T) s2 += st.cum[(size_t)b * T + src] * wcv[(size_t)tap * Fw + ff];
        }
        fl[((size_t)b * T + j) * Fw + ff] = s2;
      }
  gemm(fl.data(), B * T, Fw, Fw, wl.data(), A, nullptr, loc.data(), A);
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < T; ++j) {
      const size_t r = (size_t)b * T + j;
      float e = 0.f;
      for (int k = 0; k < A; ++k) e += va[k] * std::tanh(c->keys[r * A + k] + q[(size_t)b * A + k] + loc[r * A + k] + ba[k]);
      en[r] = e;
    }
  std::vector<float> ctx((size_t)B * D, 0.f);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    const int len = c->lens[b], pm = st.max_att[b], win = cfg.attention_win_size;
    std::vector<float> sc(T);
    float mx = -INFINITY;
    for (int j = 0; j < T; ++j) {
      float e = en[(size_t)b * T + j];
      if (cfg.synthesis_constraint) {  // attention.py:202-215
        const bool masked = cfg.constraint_monotonic ? (j < pm || j >= pm + win)
                                                     : (j < pm - (win / 2 + (win % 2 != 0 ? 1 : 0)) || j >= pm + win / 2);
        if (masked) e = -4294967296.0f;
      }
      if (cfg.mask_encoder && j >= len) e = -INFINITY;
      sc[j] = e;
      mx = std::max(mx, e);
    }
    float sum = 0.f;
    if (cfg.smoothing)  // _smoothing_normalization (attention.py:71-80): sigmoid(e) / sum sigmoid(e)
      for (int j = 0; j < T; ++j) sum += (sc[j] = 1.f / (1.f + std::exp(-sc[j])));
    else
      for (int j = 0; j < T; ++j) sum += (sc[j] = std::exp(sc[j] - mx));
    float best = -INFINITY;
    int bi = 0;
    for (int j = 0; j < T; ++j) {
      const float a = sc[j] / sum;
      if (align) align[(size_t)b * T + j] = a;
      st.cum[(size_t)b * T + j] = cfg.cumulative_weights ? a + st.cum[(size_t)b * T + j] : a;
      if (a > best) {
        best = a;
        bi = j;
      }
      const float* v = &c->values[((size_t)b * T + j) * D];
      float* cx = &ctx[(size_t)b * D];
      for (int d = 0; d < D; ++d) cx[d] += a * v[d];
    }
    st.max_att[b] = bi;
  }
  st.ctx.swap(ctx);
  // frame / stop projections on [h2_new, context] (Architecture_wrappers.py:243-247): r frames and r
  // stop tokens per step (FrameProjection(num_mels * r), StopProjection(shape=r), tacotron.py:322-324)
  const int r = cfg.outputs_per_step, NF = nm * r;
  std::vector<float> pin((size_t)B * (H + D));
  for (int b = 0; b < B; ++b) {
    std::memcpy(&pin[(size_t)b * (H + D)], &o2[(size_t)b * H], sizeof(float) * H);
    std::memcpy(&pin[(size_t)b * (H + D) + H], &st.ctx[(size_t)b * D], sizeof(float) * D);
  }
  const std::string fp = "decoder/linear_transform_projection/projection_linear_transform_projection/";
  const std::string sp = "decoder/stop_token_projection/projection_stop_token_projection/";
  gemm(pin.data(), B, H + D, H + D, W(c, fp + "kernel", {H + D, NF}).data(), NF, W(c, fp + "bias", {NF}).data(),
       frame, NF);
  gemm(pin.data(), B, H + D, H + D, W(c, sp + "kernel", {H + D, r}).data(), r, W(c, sp + "bias", {r}).data(), stop, r);
  for (int i = 0; i < B * r; ++i) stop[i] = sigm(stop[i]);
}

DecState zero_state(const tt2_ctx* c) {
  DecState st;
  const size_t B = c->B, H = c->H;
  st.h1.assign(B * H, 0.f); st.c1.assign(B * H, 0.f); st.h2.assign(B * H, 0.f); st.c2.assign(B * H, 0.f);
  st.ctx.assign(B * c->Dm, 0.f);
  st.cum.assign(B * c->T_in, 0.f);
  st.max_att.assign(B, 0);
  return st;
}

void check_finalized(tt2_ctx* c) {
  const auto& cfg = c->cfg;
  // the variables whose shapes fix the model's widths, checked before the first call (every other
  // variable is checked by name and shape where it is used)
  (void)W(c, "inputs_embedding", {cfg.n_symbols, c->E});
  (void)W(c, "memory_layer/kernel", {c->Dm, c->A});
  (void)W(c, "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel", {c->P + c->Dm + c->H, 4 * c->H});
  (void)W(c, "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/kernel", {2 * c->H, 4 * c->H});
  (void)W(c, "postnet_projection/projection_postnet_projection/kernel", {c->PC, c->nm});
}

}  // namespace

extern "C" {

const char* tt2_last_error(void) { return g_err.c_str(); }
const char* tt2_version(void) { return "libtt2_cpu 0.1 host fp32 (OpenMP)"; }

void tt2_default_config(tt2_config* c, int max_batch, int max_T_in, int max_T_ref, int max_iters) {
  std::memset(c, 0, sizeof(*c));
  c->num_mels = 80; c->n_symbols = 66; c->embedding_dim = 512; c->enc_conv_num_layers = 3;
  c->enc_conv_kernel_size = 5; c->enc_conv_channels = 512; c->encoder_lstm_units = 256;
  c->attention_dim = 128; c->attention_filters = 32; c->attention_kernel = 31; c->prenet_units = 256;
  c->decoder_lstm_units = 1024; c->postnet_num_layers = 5; c->postnet_kernel_size = 5; c->postnet_channels = 512;
  c->use_gst = 1; c->emt_only = 0; c->num_gst = 10; c->num_heads = 4; c->style_embed_depth = 256;
  c->style_att_dim = 128; c->reference_depth = 128;
  const int rf[6] = {32, 32, 64, 64, 128, 128};
  for (int i = 0; i < 6; ++i) c->reference_filters[i] = rf[i];
  c->zoneout = 0.1f; c->max_abs_value = 4.f; c->lower_bound_decay = 0.1f; c->symmetric_mels = 1;
  c->clip_outputs = 1; c->stop_at_any = 0; c->mask_encoder = 1; c->cumulative_weights = 1;
  c->synthesis_constraint = 0; c->constraint_monotonic = 0; c->attention_win_size = 7;
  c->max_batch = max_batch; c->max_T_in = max_T_in; c->max_T_ref = max_T_ref; c->max_iters = max_iters;
  c->emt_attn = 0; c->emt_ref_gru = 0; c->n_emt = 4; c->style_mode = 0;
  c->smoothing = 0; c->outputs_per_step = 1;
}

tt2_status tt2_create(const tt2_config* cfg, int hip_device, tt2_ctx** out) {
  return guard([&] {
    CK(cfg && out, TT2_ERR_INVALID_ARG, "tt2_create: null argument");
    (void)hip_device;  // host backend: the device index is ignored
    *out = nullptr;
    CK(cfg->max_batch >= 1 && cfg->max_T_in >= 1 && cfg->max_iters >= 1, TT2_ERR_INVALID_ARG, "capacities must be >= 1");
    CK(cfg->emt_attn == 0, TT2_ERR_INVALID_ARG, "the CPU backend builds the Tacotron model only (emt_attn = 0)");

    CK(cfg->attention_filters <= 64, TT2_ERR_INVALID_ARG, "attention_filters must be <= 64");
    CK(cfg->outputs_per_step >= 1 && cfg->outputs_per_step <= 8, TT2_ERR_INVALID_ARG, "outputs_per_step must be in [1, 8]");
    auto c = std::make_unique<tt2_ctx>();
    c->cfg = *cfg;
    c->nm = cfg->num_mels; c->E = cfg->embedding_dim; c->Cenc = cfg->enc_conv_channels; c->U = cfg->encoder_lstm_units;
    c->A = cfg->attention_dim; c->F = cfg->attention_filters; c->KL = cfg->attention_kernel; c->P = cfg->prenet_units;
    c->H = cfg->decoder_lstm_units; c->PC = cfg->postnet_channels;
    // style path (tacotron.py:236-308): use_gst=False takes the reference embeddings themselves
    c->style_mode = (!cfg->use_gst && cfg->style_mode == 0) ? 1 : cfg->style_mode;
    CK(c->style_mode >= 0 && c->style_mode <= 2, TT2_ERR_INVALID_ARG, "style_mode must be 0..2");
    CK(!(c->style_mode == 2 && cfg->emt_only), TT2_ERR_INVALID_ARG, "must provide speaker reference to use AdaIn");
    c->nref = c->style_mode == 2 ? 1 : (cfg->emt_only ? 1 : 2);
    c->nmel = c->style_mode == 2 ? 2 : c->nref;
    c->SW = c->style_mode == 0 ? c->nref * cfg->style_embed_depth : 128 * c->nref;
    c->Dm = 2 * c->U + c->SW;
    *out = c.release();
  });
}

void tt2_destroy(tt2_ctx* c) {
  g_pack.clear();
  delete c;
}

tt2_status tt2_load_tensor(tt2_ctx* c, const char* name, const float* host, const int64_t* shape, int ndim) {
  return guard([&] {
    CK(c, TT2_ERR_INVALID_ARG, "null ctx");
    g_pack.clear();
    put(c->wm, name, host, shape, ndim);
    c->finalized = false;
  });
}

tt2_status tt2_finalize_weights(tt2_ctx* c) {
  return guard([&] {
    CK(c, TT2_ERR_INVALID_ARG, "null ctx");
    check_finalized(c);
    c->finalized = true;
  });
}

tt2_status tt2_encode(tt2_ctx* c, const int32_t* ids, const int32_t* lengths, int B, int T_in, const float* ref_emt,
                      int T_ref_emt, const float* ref_spk, int T_ref_spk, float* memory_out, float* style_out) {
  return guard([&] {
    CK(c && ids && lengths, TT2_ERR_INVALID_ARG, "tt2_encode: null argument");
    CK(ref_emt && (c->nmel < 2 || ref_spk), TT2_ERR_INVALID_ARG, "must provide references");  // tacotron.py:66-67
    const float* refs[2] = {ref_emt, ref_spk};
    const int trs[2] = {T_ref_emt, T_ref_spk};
    encode(c, ids, lengths, B, T_in, refs, trs);
    if (memory_out) std::memcpy(memory_out, c->values.data(), sizeof(float) * c->values.size());
    if (style_out) std::memcpy(style_out, c->style.data(), sizeof(float) * (size_t)B * c->SW);
  });
}

tt2_status tt2_decode(tt2_ctx* c, int max_iters, const uint8_t* prenet_masks, uint64_t seed, const float* targets,
                      int T_targets, float* frames, float* stop, float* align, int32_t* n_steps) {
  return guard([&] {
    CK(c && frames && stop && n_steps, TT2_ERR_INVALID_ARG, "tt2_decode: null argument");
    CK(c->encoded, TT2_ERR_STATE, "tt2_decode called before tt2_encode");
    CK(max_iters >= 1 && max_iters <= c->cfg.max_iters, TT2_ERR_SHAPE_MISMATCH, "max_iters exceeds capacity");
    const int B = c->B, T = c->T_in, nm = c->nm, P = c->P, r = c->cfg.outputs_per_step;
    CK(!targets || T_targets >= r, TT2_ERR_INVALID_ARG, "targets given with T_targets < outputs_per_step");
    std::vector<uint8_t> gm;
    if (!prenet_masks) {  // the device RNG's stream (rng.h), identical bits
      gm.resize((size_t)max_iters * 2 * B * P);
      for (size_t i = 0; i < gm.size(); ++i) gm[i] = prenet_keep_bit((long)i, seed);
      prenet_masks = gm.data();
    }
    DecState st = zero_state(c);
    const size_t NF = (size_t)nm * r, fs = (size_t)max_iters * r;  // frames per step / per row
    std::vector<float> fin((size_t)B * nm, 0.f), fr(B * NF), sp((size_t)B * r), al((size_t)B * T);
    c->frames.assign(B * fs * nm, 0.f);
    // GTA: len(targets[:, r-1::r]) = T_targets / r steps (helpers.py:78-81)
    const int n_limit = targets ? std::min(max_iters, T_targets / r) : max_iters;
    int t = 0;
    for (; t < n_limit; ++t) {
      dec_step(c, fin.data(), prenet_masks + (size_t)t * 2 * B * P, st, fr.data(), sp.data(), al.data());
      for (int b = 0; b < B; ++b) {
        std::memcpy(&frames[(b * fs + (size_t)t * r) * nm], &fr[b * NF], sizeof(float) * NF);
        std::memcpy(&c->frames[(b * fs + (size_t)t * r) * nm], &fr[b * NF], sizeof(float) * NF);
        for (int i = 0; i < r; ++i) stop[b * fs + (size_t)t * r + i] = sp[(size_t)b * r + i];
        if (align)
          for (int j = 0; j < T; ++j) align[((size_t)b * T + j) * max_iters + t] = al[(size_t)b * T + j];
      }
      if (targets) {  // GTA TacoTrainingHelper, ratio 1: frame t·r + r - 1 (helpers.py:78, 126-129)
        for (int b = 0; b < B; ++b)
          std::memcpy(&fin[(size_t)b * nm], &targets[((size_t)b * T_targets + (size_t)t * r + r - 1) * nm],
                      sizeof(float) * nm);
        continue;
      }
      // TacoTestHelper stop rule (helpers.py:40-54): finished = round(stop) [B, r]; reduce_all over the
      // batch axis first, then any (stop_at_any) / all over the step's r frames
      bool any_f = false, all_f = true;
      for (int i = 0; i < r; ++i) {
        int fin_rows = 0;
        for (int b = 0; b < B; ++b) fin_rows += std::nearbyint(sp[(size_t)b * r + i]) == 1.f;
        any_f |= fin_rows == B;
        all_f &= fin_rows == B;
      }
      if (c->cfg.stop_at_any == 2 ? false : (c->cfg.stop_at_any ? any_f : all_f)) {
        ++t;
        break;
      }
      for (int b = 0; b < B; ++b)  // the step's last frame is the next input (helpers.py:57)
        std::memcpy(&fin[(size_t)b * nm], &fr[b * NF + NF - nm], sizeof(float) * nm);
    }
    c->n_steps = t;
    c->max_iters_last = max_iters;
    *n_steps = t;
    c->decoded = true;
  });
}

tt2_status tt2_prenet_keep_bits(uint64_t seed, int max_iters, int B, int prenet_units, uint8_t* out) {
  return guard([&] {
    CK(out && max_iters >= 1 && B >= 1 && prenet_units >= 1, TT2_ERR_INVALID_ARG, "tt2_prenet_keep_bits: bad argument");
    const long n = (long)max_iters * 2 * B * prenet_units;
    for (long i = 0; i < n; ++i) out[i] = prenet_keep_bit(i, seed);
  });
}

tt2_status tt2_decoder_step(tt2_ctx* c, const float* frame_in, const uint8_t* prenet_masks,
                            const tt2_decoder_state* in, tt2_decoder_state* out, float* frame_out, float* stop_out,
                            float* alignments_out) {
  return guard([&] {
    CK(c && frame_in && prenet_masks && in && out && frame_out && stop_out, TT2_ERR_INVALID_ARG,
       "tt2_decoder_step: null argument");
    CK(c->encoded, TT2_ERR_STATE, "tt2_decoder_step called before tt2_encode");
    CK(c->cfg.outputs_per_step == 1, TT2_ERR_INVALID_ARG, "tt2_decoder_step: outputs_per_step > 1 decodes through tt2_decode");
    const size_t B = c->B, H = c->H, D = c->Dm, T = c->T_in;
    DecState st;
    st.h1.assign(in->h1, in->h1 + B * H); st.c1.assign(in->c1, in->c1 + B * H);
    st.h2.assign(in->h2, in->h2 + B * H); st.c2.assign(in->c2, in->c2 + B * H);
    st.ctx.assign(in->attention, in->attention + B * D);
    st.cum.assign(in->alignments, in->alignments + B * T);
    st.max_att.assign(in->max_attentions, in->max_attentions + B);
    std::vector<float> al(B * T);
    dec_step(c, frame_in, prenet_masks, st, frame_out, stop_out, al.data());
    std::memcpy(out->h1, st.h1.data(), sizeof(float) * B * H); std::memcpy(out->c1, st.c1.data(), sizeof(float) * B * H);
    std::memcpy(out->h2, st.h2.data(), sizeof(float) * B * H); std::memcpy(out->c2, st.c2.data(), sizeof(float) * B * H);
    std::memcpy(out->attention, st.ctx.data(), sizeof(float) * B * D);
    std::memcpy(out->alignments, st.cum.data(), sizeof(float) * B * T);
    std::memcpy(out->max_attentions, st.max_att.data(), sizeof(int) * B);
    out->time = in->time + 1;
    if (alignments_out) std::memcpy(alignments_out, al.data(), sizeof(float) * B * T);
  });
}

tt2_status tt2_postnet(tt2_ctx* c, const float* frames_in, int B, int T, float* decoder_output, float* mel_out) {
  return guard([&] {
    CK(c && mel_out, TT2_ERR_INVALID_ARG, "tt2_postnet: null argument");
    const auto& cfg = c->cfg;
    const int nm = c->nm;
    std::vector<float> dec;
    if (!frames_in) {
      CK(c->decoded, TT2_ERR_STATE, "tt2_postnet(NULL) called before tt2_decode");
      B = c->B;
      const int r = cfg.outputs_per_step;
      T = c->n_steps * r;
      dec.resize((size_t)B * T * nm);
      for (int b = 0; b < B; ++b)
        std::memcpy(&dec[(size_t)b * T * nm], &c->frames[(size_t)b * c->max_iters_last * r * nm], sizeof(float) * T * nm);
    } else {
      CK(B >= 1 && T >= 1, TT2_ERR_INVALID_ARG, "tt2_postnet: B, T must be >= 1");
      dec.assign(frames_in, frames_in + (size_t)B * T * nm);
    }
    // tacotron.py:362-381: clip, Postnet (4 x conv tanh + conv linear, BN after each), projection,
    // residual, clip
    const float lo = cfg.symmetric_mels ? -cfg.max_abs_value - cfg.lower_bound_decay : -cfg.lower_bound_decay;
    const float hi = cfg.max_abs_value;
    if (cfg.clip_outputs)
      for (auto& v : dec) v = std::min(std::max(v, lo), hi);
    std::vector<float> x(dec), y;
    int cin = nm;
    for (int i = 1; i <= cfg.postnet_num_layers; ++i) {
      const std::string s = "postnet_convolutions/conv_layer_" + std::to_string(i) + "_postnet_convolutions/";
      y.assign((size_t)B * T * c->PC, 0.f);
      conv1d_bn(x.data(), B, T, cin, W(c, s + "conv1d/kernel", {cfg.postnet_kernel_size, cin, c->PC}),
                cfg.postnet_kernel_size, c->PC, W(c, s + "conv1d/bias", {c->PC}), bn_consts(c->wm, TP + s, c->PC),
                i < cfg.postnet_num_layers ? 2 : 0, y.data());
      x.swap(y);
      cin = c->PC;
    }
    const std::string pp = "postnet_projection/projection_postnet_projection/";
    gemm(x.data(), B * T, c->PC, c->PC, W(c, pp + "kernel", {c->PC, nm}).data(), nm, W(c, pp + "bias", {nm}).data(),
         mel_out, nm);
    for (size_t i = 0; i < dec.size(); ++i) {
      float v = dec[i] + mel_out[i];
      if (cfg.clip_outputs) v = std::min(std::max(v, lo), hi);
      mel_out[i] = v;
    }
    if (decoder_output) std::memcpy(decoder_output, dec.data(), sizeof(float) * dec.size());
  });
}

}  // extern "C"

// =====================================================================================================
// WaveNet
// =====================================================================================================
struct tt2_wn_ctx {
  tt2_wn_config cfg;
  WeightMap wm;
  bool finalized = false;
};

namespace {

const char* WP = "WaveNet_model/inference/";

const std::vector<float>& WW(const tt2_wn_ctx* c, const std::string& n, std::vector<int64_t> s) {
  return need(c->wm, WP + n, std::move(s));
}

inline float up_act(const tt2_wn_config& cfg, float v) {
  if (cfg.upsample_activation == 1) return std::max(v, 0.f);
  if (cfg.upsample_activation == 2) return std::max(v, cfg.leaky_alpha * v);
  return v;
}

// Conditioning upsampling network (wavenet.py:163-203, applied at :782-803) on one row,
// channels-first x [F][T] -> [F][T·Πs]; every upsample_type.
std::vector<float> upsample(const tt2_wn_ctx* c, std::vector<float> x, int F, int T) {
  const auto& cfg = c->cfg;
  const int KF = cfg.freq_axis_kernel_size, pf = (KF - 1) / 2;
  const int ut = cfg.upsample_type;
  if (ut == 4) {  // NearestNeighbor: repeat x hop (modules.py:524-536)
    int hop = 1;
    for (int i = 0; i < cfg.n_upsample; ++i) hop *= cfg.upsample_scales[i];
    std::vector<float> y((size_t)F * T * hop);
    for (int f = 0; f < F; ++f)
      for (int t = 0; t < T * hop; ++t) y[(size_t)f * T * hop + t] = x[(size_t)f * T + t / hop];
    return y;
  }
  const char* names[4] = {"ConvTranspose2D", "ConvTranspose1D", "ResizeConvolution", "SubPixelConvolution"};
  for (int i = 0; i < cfg.n_upsample; ++i) {
    const int s = cfg.upsample_scales[i];
    const std::string sc = "local_conditioning_upsampling_" + std::to_string(i + 1) + "/" + names[ut] + "_layer_" +
                           std::to_string(i) + "/";
    const int To = T * s;
    std::vector<float> y((size_t)F * To, 0.f);
    auto X = [&](int f, int t) { return (f < 0 || f >= F || t < 0 || t >= T) ? 0.f : x[(size_t)f * T + t]; };
    if (ut == 0) {  // ConvTranspose2D 1->1, kernel (KF, s), stride (1, s), 'same'
      const auto& K = WW(c, sc + "kernel", {KF, s, 1, 1});
      const float b = WW(c, sc + "bias", {1})[0];
      for (int f = 0; f < F; ++f)
        for (int t = 0; t < T; ++t)
          for (int j = 0; j < s; ++j) {
            float acc = 0.f;
            for (int d = 0; d < KF; ++d) acc += X(f + pf - d, t) * K[(size_t)d * s + j];
            y[(size_t)f * To + t * s + j] = up_act(cfg, acc + b);
          }
    } else if (ut == 1) {  // ConvTranspose1D F->F, kernel (1, s) == stride: no overlap
      const auto& K = WW(c, sc + "kernel", {1, s, F, F});
      const auto& b = WW(c, sc + "bias", {F});
      for (int o = 0; o < F; ++o)
        for (int t = 0; t < T; ++t)
          for (int j = 0; j < s; ++j) {
            float acc = b[o];
            for (int ci = 0; ci < F; ++ci) acc += x[(size_t)ci * T + t] * K[((size_t)j * F + o) * F + ci];
            y[(size_t)o * To + t * s + j] = up_act(cfg, acc);
          }
    } else if (ut == 2) {  // NN resize x s on time, then Conv2D 1->1 kernel (KF, s) 'same'
      const auto& K = WW(c, sc + "kernel", {KF, s, 1, 1});
      const float b = WW(c, sc + "bias", {1})[0];
      const int pt = (s - 1) / 2;
      for (int f = 0; f < F; ++f)
        for (int t = 0; t < To; ++t) {
          float acc = 0.f;
          for (int d = 0; d < KF; ++d)
            for (int qq = 0; qq < s; ++qq) {
              const int ff = f + d - pf, tt = t + qq - pt;
              if (ff < 0 || ff >= F || tt < 0 || tt >= To) continue;
              acc += x[(size_t)ff * T + tt / s] * K[(size_t)d * s + qq];
            }
          y[(size_t)f * To + t] = up_act(cfg, acc + b);
        }
    } else {  // SubPixel: Conv2D 1->s kernel (KF, 3) 'same', periodic shuffle (modules.py:539-654)
      const auto& K = WW(c, sc + "kernel", {KF, 3, 1, s});
      const auto& b = WW(c, sc + "bias", {s});
      for (int f = 0; f < F; ++f)
        for (int w = 0; w < T; ++w)
          for (int k = 0; k < s; ++k) {
            const int kk = cfg.NN_init ? k : 0;  // NN_init=False: every channel uses channel 0's kernel
            float acc = 0.f;
            for (int d = 0; d < KF; ++d)
              for (int qq = 0; qq < 3; ++qq) acc += X(f + d - pf, w + qq - 1) * K[((size_t)d * 3 + qq) * s + kk];
            y[(size_t)f * To + w * s + k] = up_act(cfg, acc + b[k]);
          }
    }
    x.swap(y);
    T = To;
  }
  return x;
}

}  // namespace

extern "C" {

void tt2_wn_default_config(tt2_wn_config* c, int max_batch, int64_t max_samples) {
  std::memset(c, 0, sizeof(*c));
  c->layers = 24; c->stacks = 4; c->residual_channels = 64; c->gate_channels = 128; c->skip_out_channels = 64;
  c->kernel_size = 3; c->cin_channels = 80; c->out_channels = 30; c->legacy = 1; c->residual_legacy = 1;
  c->log_scale_min = (float)std::log(1e-14); c->n_upsample = 3;
  c->upsample_scales[0] = 5; c->upsample_scales[1] = 5; c->upsample_scales[2] = 11;
  c->freq_axis_kernel_size = 3; c->max_batch = max_batch; c->max_samples = max_samples;
  c->upsample_type = 0; c->upsample_activation = 1; c->leaky_alpha = 0.4f; c->NN_init = 1;
  c->log_scale_min_gauss = (float)std::log(1e-7);
}

tt2_status tt2_wn_create(const tt2_wn_config* cfg, int hip_device, tt2_wn_ctx** out) {
  return guard([&] {
    CK(cfg && out, TT2_ERR_INVALID_ARG, "tt2_wn_create: null argument");
    (void)hip_device;
    *out = nullptr;
    CK(cfg->gin_channels <= 0, TT2_ERR_INVALID_ARG, "global conditioning is GPU-only (libtt2.so)");
    CK(cfg->input_type != 2 && cfg->cin_channels > 0, TT2_ERR_INVALID_ARG,
       "mulaw-quantize input and unconditional synthesis are GPU-only (libtt2.so)");
    CK(cfg->kernel_size >= 1 && cfg->layers >= 1 && cfg->stacks >= 1 && cfg->layers % cfg->stacks == 0,
       TT2_ERR_INVALID_ARG, "layers must be a multiple of stacks");
    CK(cfg->upsample_type >= 0 && cfg->upsample_type <= 4, TT2_ERR_INVALID_ARG, "upsample_type must be 0..4");
    CK(cfg->out_channels == 2 || cfg->out_channels % 3 == 0, TT2_ERR_INVALID_ARG, "out_channels: 2 or 3*nr_mix");
    auto c = std::make_unique<tt2_wn_ctx>();
    c->cfg = *cfg;
    *out = c.release();
  });
}

void tt2_wn_destroy(tt2_wn_ctx* c) {
  g_pack.clear();
  delete c;
}

tt2_status tt2_wn_load_tensor(tt2_wn_ctx* c, const char* name, const float* host, const int64_t* shape, int ndim) {
  return guard([&] {
    CK(c, TT2_ERR_INVALID_ARG, "null ctx");
    g_pack.clear();
    put(c->wm, name, host, shape, ndim);
    c->finalized = false;
  });
}

tt2_status tt2_wn_finalize(tt2_wn_ctx* c) {
  return guard([&] {
    CK(c, TT2_ERR_INVALID_ARG, "null ctx");
    const auto& cfg = c->cfg;
    (void)WW(c, "input_convolution/kernel", {1, 1, cfg.residual_channels});
    (void)WW(c, "skip_convolutions/final_convolution_2/kernel", {1, cfg.skip_out_channels, cfg.out_channels});
    c->finalized = true;
  });
}

// WaveNet.incremental (wavenet.py:724-911) with the fast-WaveNet queues (modules.py:270-297)
tt2_status tt2_wn_generate(tt2_wn_ctx* c, const float* cond, int B, int T_f, const float* u_mix, const float* u_log,
                           uint64_t seed, const float* teacher, float* wav_out, int32_t* mix_idx_out, float* logits_out,
                           float* upsampled_out) {
  return guard([&] {
    CK(c && cond && wav_out, TT2_ERR_INVALID_ARG, "tt2_wn_generate: null argument");
    CK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_wn_finalize not called");
    const auto& cfg = c->cfg;
    CK(B >= 1 && B <= cfg.max_batch && T_f >= 1, TT2_ERR_SHAPE_MISMATCH, "batch exceeds capacity");
    int hop = 1;
    for (int i = 0; i < cfg.n_upsample; ++i) hop *= cfg.upsample_scales[i];
    const long T = (long)T_f * hop;
    CK(T <= cfg.max_samples, TT2_ERR_SHAPE_MISMATCH, "T_f * hop exceeds max_samples");
    const int R = cfg.residual_channels, G = cfg.gate_channels, G2 = G / 2, S = cfg.skip_out_channels,
              Cin = cfg.cin_channels, C = cfg.out_channels, L = cfg.layers, per = L / cfg.stacks, kw = cfg.kernel_size;
    const bool gauss = C == 2;
    const int nr = gauss ? 0 : C / 3;
    const float SQH = std::sqrt(0.5f);
    const auto& fk = WW(c, "input_convolution/kernel", {1, 1, R});
    const auto& fb = WW(c, "input_convolution/bias", {R});
    struct Layer {
      int d;
      const float *k, *b, *kc, *bc, *ks, *bs, *ko, *bo;
    };
    std::vector<Layer> ly(L);
    for (int l = 0; l < L; ++l) {
      const std::string s = "ResidualConv1DGLU_" + std::to_string(l) + "/";
      auto sc = [&](const char* kind) {
        return s + "residual_block_" + kind + "_conv_ResidualConv1DGLU_" + std::to_string(l) + "/";
      };
      ly[l].d = 1 << (l % per);
      ly[l].k = WW(c, sc("causal") + "kernel", {kw, R, G}).data();
      ly[l].b = WW(c, sc("causal") + "bias", {G}).data();
      ly[l].kc = WW(c, sc("cin") + "kernel", {1, Cin, G}).data();
      ly[l].bc = WW(c, sc("cin") + "bias", {G}).data();
      ly[l].ks = WW(c, sc("skip") + "kernel", {1, G2, S}).data();
      ly[l].bs = WW(c, sc("skip") + "bias", {S}).data();
      ly[l].ko = WW(c, sc("out") + "kernel", {1, G2, R}).data();
      ly[l].bo = WW(c, sc("out") + "bias", {R}).data();
    }
    const auto& f1k = WW(c, "skip_convolutions/final_convolution_1/kernel", {1, S, S});
    const auto& f1b = WW(c, "skip_convolutions/final_convolution_1/bias", {S});
    const auto& f2k = WW(c, "skip_convolutions/final_convolution_2/kernel", {1, S, C});
    const auto& f2b = WW(c, "skip_convolutions/final_convolution_2/bias", {C});
    CK(!gauss || u_log, TT2_ERR_INVALID_ARG, "the CPU backend's Gaussian head needs injected N(0,1) draws (u_log)");
    // utterances are independent (the reference's batched synthesis, hparams.py:332): one OpenMP
    // thread per row; inside a row the sample chain is sequential
#pragma omp parallel for schedule(dynamic, 1) if (B > 1)
    for (int b = 0; b < B; ++b) {
      // conditioning: [T_f][Cin] -> channels-first, upsampled [Cin][T]; per layer cin conv of
      // every sample at once (one GEMM per layer)
      std::vector<float> xc((size_t)Cin * T_f);
      for (int t = 0; t < T_f; ++t)
        for (int f = 0; f < Cin; ++f) xc[(size_t)f * T_f + t] = cond[((size_t)b * T_f + t) * Cin + f];
      const std::vector<float> up = upsample(c, xc, Cin, T_f);
      if (upsampled_out) std::memcpy(upsampled_out + (size_t)b * Cin * T, up.data(), sizeof(float) * Cin * T);
      std::vector<float> ct((size_t)T * Cin);
      for (int f = 0; f < Cin; ++f)
        for (long t = 0; t < T; ++t) ct[(size_t)t * Cin + f] = up[(size_t)f * T + t];
      std::vector<std::vector<float>> cc(L);
      for (int l = 0; l < L; ++l) {
        cc[l].resize((size_t)T * G);
        gemm(ct.data(), (int)T, Cin, Cin, ly[l].kc, G, ly[l].bc, cc[l].data(), G);
      }
      // queues: layer l keeps its last (kw-1)·d + 1 inputs (modules.py:285-292)
      std::vector<std::vector<float>> q(L);
      std::vector<int> qlen(L);
      for (int l = 0; l < L; ++l) {
        qlen[l] = (kw - 1) * ly[l].d + 1;
        q[l].assign((size_t)qlen[l] * R, 0.f);
      }
      std::vector<long> head(L, 0);
      float cur = 0.f;  // initial input 0 ('raw'), wavenet.py:437-445
      std::vector<float> x(R), res(R), h(G), z(G2), sk(S), skips(S), taps((size_t)kw * R), o1(S), o2(C), xo(R);
      for (long t = 0; t < T; ++t) {
        for (int r = 0; r < R; ++r) x[r] = cur * fk[r] + fb[r];
        for (int l = 0; l < L; ++l) {
          const Layer& Ly = ly[l];
          res = x;
          // ring: slot (head) holds the newest input after this push
          head[l] = (head[l] + 1) % qlen[l];
          std::memcpy(&q[l][(size_t)head[l] * R], x.data(), sizeof(float) * R);
          for (int k = 0; k < kw; ++k) {  // taps oldest first: t - (kw-1-k)·d
            const long slot = ((head[l] - (long)(kw - 1 - k) * Ly.d) % qlen[l] + qlen[l]) % qlen[l];
            std::memcpy(&taps[(size_t)k * R], &q[l][(size_t)slot * R], sizeof(float) * R);
          }
          for (int g = 0; g < G; ++g) h[g] = Ly.b[g] + cc[l][(size_t)t * G + g];
          for (int k = 0; k < kw * R; ++k) {
            const float tv = taps[k];
            const float* w = Ly.k + (size_t)k * G;
            for (int g = 0; g < G; ++g) h[g] += tv * w[g];
          }
          for (int g = 0; g < G2; ++g) z[g] = std::tanh(h[g]) * sigm(h[G2 + g]);  // modules.py:510
          for (int s2 = 0; s2 < S; ++s2) sk[s2] = Ly.bs[s2];
          for (int r = 0; r < R; ++r) xo[r] = Ly.bo[r];
          for (int g = 0; g < G2; ++g) {
            const float zv = z[g];
            for (int s2 = 0; s2 < S; ++s2) sk[s2] += zv * Ly.ks[(size_t)g * S + s2];
            for (int r = 0; r < R; ++r) xo[r] += zv * Ly.ko[(size_t)g * R + r];
          }
          for (int r = 0; r < R; ++r) x[r] = cfg.residual_legacy ? (xo[r] + res[r]) * SQH : xo[r] + res[r];
          for (int s2 = 0; s2 < S; ++s2)
            skips[s2] = l == 0 ? sk[s2] : (cfg.legacy ? (skips[s2] + sk[s2]) * SQH : skips[s2] + sk[s2]);
        }
        for (int j = 0; j < S; ++j) o1[j] = f1b[j];
        for (int i = 0; i < S; ++i) {
          const float v = std::max(skips[i], 0.f);
          for (int j = 0; j < S; ++j) o1[j] += v * f1k[(size_t)i * S + j];
        }
        for (int j = 0; j < C; ++j) o2[j] = f2b[j];
        for (int i = 0; i < S; ++i) {
          const float v = std::max(o1[i], 0.f);
          for (int j = 0; j < C; ++j) o2[j] += v * f2k[(size_t)i * C + j];
        }
        if (logits_out) std::memcpy(logits_out + ((size_t)b * T + t) * C, o2.data(), sizeof(float) * C);
        float y;
        int kidx = 0;
        if (gauss) {  // sample_from_gaussian (gaussian.py:39-52): u_log carries the N(0,1) draws
          const float ls = std::max(o2[1], cfg.log_scale_min_gauss);
          y = std::min(std::max(o2[0] + std::exp(ls) * u_log[(size_t)t * B + b], -1.f), 1.f);
        } else {  // sample_from_discretized_mix_logistic (mixture.py:76-107)
          float best = -INFINITY;
          for (int i = 0; i < nr; ++i) {
            const double u = u_mix ? (double)u_mix[((size_t)t * B + b) * nr + i] : (double)wn_uniform(seed, t, B, b, i);
            const float v = o2[i] - (float)std::log(-std::log(u));
            if (v > best) {
              best = v;
              kidx = i;
            }
          }
          const double ul = u_log ? (double)u_log[(size_t)t * B + b] : (double)wn_uniform(seed, t, B, b, 15);
          const float noise = (float)(std::log(ul) - std::log(1.0 - ul));
          const float ls = std::max(o2[2 * nr + kidx], cfg.log_scale_min);
          y = std::min(std::max(o2[nr + kidx] + std::exp(ls) * noise, -1.f), 1.f);
        }
        wav_out[(size_t)b * T + t] = y;
        if (mix_idx_out) mix_idx_out[(size_t)b * T + t] = kidx;
        cur = teacher ? teacher[(size_t)b * T + t] : y;  // wavenet.py:876-878
      }
    }
  });
}

tt2_status tt2_wn_noise(uint64_t seed, int T, int B, int nr_mix, int gaussian, float* u_mix, float* u_log) {
  return guard([&] {
    CK(T >= 1 && B >= 1 && u_log, TT2_ERR_INVALID_ARG, "tt2_wn_noise: bad argument");
    CK(!gaussian, TT2_ERR_INVALID_ARG, "the Gaussian draws are device-only (transcendental rounding)");
    CK(u_mix && nr_mix >= 1 && nr_mix <= 14, TT2_ERR_INVALID_ARG, "tt2_wn_noise: bad nr_mix");
    for (long t = 0; t < T; ++t)
      for (int b = 0; b < B; ++b) {
        for (int i = 0; i < nr_mix; ++i) u_mix[((size_t)t * B + b) * nr_mix + i] = wn_uniform(seed, t, B, b, i);
        u_log[(size_t)t * B + b] = wn_uniform(seed, t, B, b, 15);
      }
  });
}

tt2_status tt2_mol_sample(const float* logits, const float* u_mix, const float* u_log, int n, int nr_mix,
                          float log_scale_min, float* x, int32_t* k) {
  return guard([&] {
    CK(logits && u_mix && u_log && x && k && n >= 0 && nr_mix >= 1, TT2_ERR_INVALID_ARG, "tt2_mol_sample: bad argument");
    for (int r = 0; r < n; ++r) {
      const float* lg = logits + (size_t)r * 3 * nr_mix;
      float best = -INFINITY;
      int kk = 0;
      for (int i = 0; i < nr_mix; ++i) {
        const float v = lg[i] - (float)std::log(-std::log((double)u_mix[(size_t)r * nr_mix + i]));
        if (v > best) {
          best = v;
          kk = i;
        }
      }
      const double ul = u_log[r];
      const float noise = (float)(std::log(ul) - std::log(1.0 - ul));
      const float ls = std::max(lg[2 * nr_mix + kk], log_scale_min);
      x[r] = std::min(std::max(lg[nr_mix + kk] + std::exp(ls) * noise, -1.f), 1.f);
      k[r] = kk;
    }
  });
}

}  // extern "C"
