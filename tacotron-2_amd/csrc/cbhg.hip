// CBHG post-processing network + linear projection (cbhg.h).  Every matrix product is a gemm.hip
// call (implicit-im2col conv1d loader, fused bias / activation / batch-norm / residual / clip
// epilogues); max-pooling and the highway gate are elementwise kernels; the bidirectional GRU is
// emt.hip's gru_sequence.
//
// Reference: code/tacotron/models/modules.py:110-184 (HighwayNet, CBHG), :485-497 (conv1d with
// bnorm='after'), tacotron.py:466-478 (the commented-out caller), hparams.py:181-188.
#include "cbhg.h"

#include "emt.h"

namespace tt2 {

// tf.layers.max_pooling1d(pool, strides=1, padding='same'): window [t − (pool−1)/2, +pool), padded
// positions ignored
__global__ void k_maxpool_same(const float* __restrict__ x, int T, int C, int pool, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long bt = i / C;
  const int t = (int)(bt % T);
  const long b = bt / T;
  const int t0 = t - (pool - 1) / 2;
  float m = -INFINITY;
  for (int d = 0; d < pool; ++d) {
    const int s = t0 + d;
    if (s >= 0 && s < T) m = fmaxf(m, x[(b * T + s) * C + c]);
  }
  y[i] = m;
}

// HighwayNet (modules.py:110-122): ht = x·[W_H | W_T] + [b_H | b_T]; y = relu(H)·σ(T) + x·(1 − σ(T))
__global__ void k_highway(const float* __restrict__ ht, const float* __restrict__ x, int Hu, float* __restrict__ y,
                          long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long r = i / Hu;
  const int u = (int)(i % Hu);
  const float h = fmaxf(ht[r * 2 * Hu + u], 0.f);
  const float g = 1.0f / (1.0f + expf(-ht[r * 2 * Hu + Hu + u]));
  y[i] = h * g + x[i] * (1.f - g);
}

static void up(DevBuf& d, const std::vector<float>& h) {
  d.alloc(h.size() * sizeof(float));
  TT2_HIP(hipMemcpy(d.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
}

// tf.layers.batch_normalization(training=False) constants: x·inv + (beta − mean·inv)
static void bn_up(const WeightMap& wm, const std::string& sc, int c, DevBuf& scale, DevBuf& shift) {
  const auto& g = need(wm, sc + "batch_normalization/gamma", {c}).data;
  const auto& be = need(wm, sc + "batch_normalization/beta", {c}).data;
  const auto& mu = need(wm, sc + "batch_normalization/moving_mean", {c}).data;
  const auto& v = need(wm, sc + "batch_normalization/moving_variance", {c}).data;
  std::vector<float> s(c), h(c);
  for (int i = 0; i < c; ++i) {
    s[i] = g[i] / sqrtf(v[i] + 1e-3f);
    h[i] = be[i] - mu[i] * s[i];
  }
  up(scale, s);
  up(shift, h);
}

void cbhg_load(CbhgModel& m, const WeightMap& wm, const std::string& P, int num_mels, int kernels, int conv_channels,
               int pool_size, int projection, int projection_kernel, int highway_layers, int highway_units,
               int rnn_units, int num_freq) {
  TT2_CHECK(kernels >= 1 && kernels <= 16 && highway_layers >= 0 && highway_layers <= 8 && pool_size >= 1,
            TT2_ERR_INVALID_ARG, "CBHG: 1..16 bank kernels, <= 8 highway layers");
  TT2_CHECK(rnn_units >= 1 && rnn_units <= 256, TT2_ERR_INVALID_ARG, "CBHG: rnn_units must be <= 256");
  m.on = true;
  m.nm = num_mels; m.K = kernels; m.C = conv_channels; m.pool = pool_size; m.proj = projection;
  m.kp = projection_kernel; m.nhw = highway_layers; m.Hu = highway_units; m.R = rnn_units; m.nf = num_freq;
  const std::string sc = P + "CBHG_postnet/";
  for (int k = 1; k <= m.K; ++k) {
    const std::string s2 = sc + "conv_bank/conv1d_" + std::to_string(k) + "/";
    up(m.bank_w[k - 1], need(wm, s2 + "conv1d/kernel", {k, m.nm, m.C}).data);
    up(m.bank_b[k - 1], need(wm, s2 + "conv1d/bias", {m.C}).data);
    bn_up(wm, s2, m.C, m.bank_s[k - 1], m.bank_h[k - 1]);
  }
  up(m.p1_w, need(wm, sc + "proj1/conv1d/kernel", {m.kp, m.K * m.C, m.proj}).data);
  up(m.p1_b, need(wm, sc + "proj1/conv1d/bias", {m.proj}).data);
  bn_up(wm, sc + "proj1/", m.proj, m.p1_s, m.p1_h);
  up(m.p2_w, need(wm, sc + "proj2/conv1d/kernel", {m.kp, m.proj, m.nm}).data);
  up(m.p2_b, need(wm, sc + "proj2/conv1d/bias", {m.nm}).data);
  bn_up(wm, sc + "proj2/", m.nm, m.p2_s, m.p2_h);
  if (m.nm != m.Hu) {
    up(m.dn_w, need(wm, sc + "dense/kernel", {m.nm, m.Hu}).data);
    up(m.dn_b, need(wm, sc + "dense/bias", {m.Hu}).data);
  }
  const int Hu = m.Hu, R = m.R;
  for (int i = 0; i < m.nhw; ++i) {  // [W_H | W_T] side by side: one GEMM per layer
    const std::string s2 = sc + "CBHG_postnet_highwaynet_" + std::to_string(i + 1) + "/";
    const auto& wh = need(wm, s2 + "H/kernel", {Hu, Hu}).data;
    const auto& wt = need(wm, s2 + "T/kernel", {Hu, Hu}).data;
    const auto& bh = need(wm, s2 + "H/bias", {Hu}).data;
    const auto& bt = need(wm, s2 + "T/bias", {Hu}).data;
    std::vector<float> w((size_t)Hu * 2 * Hu), b(2 * Hu);
    for (int r = 0; r < Hu; ++r)
      for (int c = 0; c < Hu; ++c) {
        w[(size_t)r * 2 * Hu + c] = wh[(size_t)r * Hu + c];
        w[(size_t)r * 2 * Hu + Hu + c] = wt[(size_t)r * Hu + c];
      }
    for (int c = 0; c < Hu; ++c) {
      b[c] = bh[c];
      b[Hu + c] = bt[c];
    }
    up(m.hw_w[i], w);
    up(m.hw_b[i], b);
  }
  {  // BiGRU: x rows of both directions' gates + candidate kernels in one [Hu][2·3R] matrix
    std::vector<float> wx((size_t)Hu * 6 * R), bx(6 * R), whg, whc;
    const char* names[2] = {"fw/CBHG_postnet_forward_RNN/", "bw/CBHG_postnet_backward_RNN/"};
    for (int d = 0; d < 2; ++d) {
      const std::string s2 = sc + "bidirectional_rnn/" + names[d];
      const auto& kg = need(wm, s2 + "gates/kernel", {Hu + R, 2 * R}).data;
      const auto& bg = need(wm, s2 + "gates/bias", {2 * R}).data;
      const auto& kc = need(wm, s2 + "candidate/kernel", {Hu + R, R}).data;
      const auto& bc = need(wm, s2 + "candidate/bias", {R}).data;
      const size_t o = (size_t)d * 3 * R;
      for (int k = 0; k < Hu; ++k) {
        for (int j = 0; j < 2 * R; ++j) wx[(size_t)k * 6 * R + o + j] = kg[(size_t)k * 2 * R + j];
        for (int j = 0; j < R; ++j) wx[(size_t)k * 6 * R + o + 2 * R + j] = kc[(size_t)k * R + j];
      }
      for (int j = 0; j < 2 * R; ++j) bx[o + j] = bg[j];
      for (int j = 0; j < R; ++j) bx[o + 2 * R + j] = bc[j];
      whg.insert(whg.end(), kg.begin() + (size_t)Hu * 2 * R, kg.end());
      whc.insert(whc.end(), kc.begin() + (size_t)Hu * R, kc.end());
    }
    up(m.gx_w, wx);
    up(m.gx_b, bx);
    up(m.g_whg, whg);
    up(m.g_whc, whc);
  }
  const std::string ps = P + "cbhg_linear_specs_projection/projection_cbhg_linear_specs_projection/";
  up(m.pj_w, need(wm, ps + "kernel", {2 * R, m.nf}).data);
  up(m.pj_b, need(wm, ps + "bias", {m.nf}).data);
}

void cbhg_linear(CbhgModel& m, const float* mels, int B, int T, float* linear, float* kpart, long kpart_floats,
                 hipStream_t s) {
  TT2_CHECK(m.on, TT2_ERR_STATE, "CBHG weights not loaded (tt2_config.predict_linear = 0)");
  const long BT = (long)B * T;
  const int KC = m.K * m.C;
  m.bank.alloc(sizeof(float) * BT * KC);
  m.pool_out.alloc(sizeof(float) * BT * KC);
  m.p1.alloc(sizeof(float) * BT * m.proj);
  for (auto& h : m.hw) h.alloc(sizeof(float) * BT * std::max(m.Hu, m.nm));
  m.ht.alloc(sizeof(float) * BT * 2 * m.Hu);
  m.xg.alloc(sizeof(float) * BT * 6 * m.R);
  m.gru.alloc(sizeof(float) * BT * 2 * m.R);
  // conv1d over [B][T][Cin] 'same' (pad (k-1)/2 left) with act + BN (+ residual) epilogue
  auto conv = [&](const float* x, int Cin, int kw, const DevBuf& w, const DevBuf& b, const DevBuf& sc,
                  const DevBuf& sh, int N, int act, float* out, long ldc, const float* res) {
    GemmArgs g;
    g.M = (int)BT; g.N = N; g.K = kw * Cin; g.a_mode = A_CONV1D; g.A = x;
    g.T = T; g.C = Cin; g.kw = kw; g.pad = (kw - 1) / 2; g.xs_b = (long)T * Cin; g.xs_t = Cin;
    g.Bw = w.as<float>(); g.ldb = N; g.Cout = out; g.ldc = ldc;
    g.bias = b.as<float>(); g.act = act; g.bn_scale = sc.as<float>(); g.bn_shift = sh.as<float>();
    g.residual = res; g.ldr = N;
    g.kpart = kpart; g.kpart_floats = kpart_floats;
    gemm(g, s);
  };
  // conv bank: kernel sizes 1..K, ReLU then BN, concatenated on channels (modules.py:146-152)
  for (int k = 1; k <= m.K; ++k)
    conv(mels, m.nm, k, m.bank_w[k - 1], m.bank_b[k - 1], m.bank_s[k - 1], m.bank_h[k - 1], m.C, ACT_RELU,
         m.bank.as<float>() + (size_t)(k - 1) * m.C, KC, nullptr);
  {
    const long n = BT * KC;
    hipLaunchKernelGGL(k_maxpool_same, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, m.bank.as<float>(), T, KC,
                       m.pool, m.pool_out.as<float>(), n);
    TT2_HIP(hipGetLastError());
  }
  conv(m.pool_out.as<float>(), KC, m.kp, m.p1_w, m.p1_b, m.p1_s, m.p1_h, m.proj, ACT_RELU, m.p1.as<float>(), m.proj,
       nullptr);
  // proj2 (linear) + BN + the residual with the input (modules.py:162-166)
  float* h = m.hw[0].as<float>();
  conv(m.p1.as<float>(), m.proj, m.kp, m.p2_w, m.p2_b, m.p2_s, m.p2_h, m.nm, ACT_NONE, h, m.nm, mels);
  if (m.nm != m.Hu) {  // dense to the highway width (modules.py:168-170)
    GemmArgs g;
    g.M = (int)BT; g.N = m.Hu; g.K = m.nm; g.A = h; g.lda = m.nm;
    g.Bw = m.dn_w.as<float>(); g.ldb = m.Hu; g.Cout = m.hw[1].as<float>(); g.ldc = m.Hu; g.bias = m.dn_b.as<float>();
    g.kpart = kpart; g.kpart_floats = kpart_floats;
    gemm(g, s);
    h = m.hw[1].as<float>();
  }
  for (int i = 0; i < m.nhw; ++i) {
    GemmArgs g;
    g.M = (int)BT; g.N = 2 * m.Hu; g.K = m.Hu; g.A = h; g.lda = m.Hu;
    g.Bw = m.hw_w[i].as<float>(); g.ldb = 2 * m.Hu; g.Cout = m.ht.as<float>(); g.ldc = 2 * m.Hu;
    g.bias = m.hw_b[i].as<float>();
    g.kpart = kpart; g.kpart_floats = kpart_floats;
    gemm(g, s);
    float* o = (h == m.hw[0].as<float>()) ? m.hw[1].as<float>() : m.hw[0].as<float>();
    const long n = BT * m.Hu;
    hipLaunchKernelGGL(k_highway, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, m.ht.as<float>(), h, m.Hu, o, n);
    TT2_HIP(hipGetLastError());
    h = o;
  }
  {  // bidirectional GRU over every frame (input_lengths None, modules.py:176-183)
    GemmArgs g;
    g.M = (int)BT; g.N = 6 * m.R; g.K = m.Hu; g.A = h; g.lda = m.Hu;
    g.Bw = m.gx_w.as<float>(); g.ldb = 6 * m.R; g.Cout = m.xg.as<float>(); g.ldc = 6 * m.R; g.bias = m.gx_b.as<float>();
    g.kpart = kpart; g.kpart_floats = kpart_floats;
    gemm(g, s);
    gru_sequence(m.xg.as<float>(), B, T, m.R, 2, m.g_whg.as<float>(), m.g_whc.as<float>(), 0, nullptr, nullptr,
                 m.gru.as<float>(), s);
  }
  GemmArgs g;  // FrameProjection(num_freq) + clip (tacotron.py:475-481)
  g.M = (int)BT; g.N = m.nf; g.K = 2 * m.R; g.A = m.gru.as<float>(); g.lda = 2 * m.R;
  g.Bw = m.pj_w.as<float>(); g.ldb = m.nf; g.Cout = linear; g.ldc = m.nf; g.bias = m.pj_b.as<float>();
  g.clip = m.clip; g.clip_lo = m.clip_lo; g.clip_hi = m.clip_hi;
  g.kpart = kpart; g.kpart_floats = kpart_floats;
  gemm(g, s);
}

}  // namespace tt2
