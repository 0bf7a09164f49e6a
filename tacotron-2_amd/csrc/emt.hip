// Tacotron_emt_attn: reference-encoder outputs, emotion attention per decoder step (emt.h).
//
// Reference: code/tacotron/models/{tacotron_emt_attn.py:198-285, modules.py:9-64 (all_outputs),
// attention.py:230-260 (SimpleBahdanauAttention), multihead_attention.py:35-132,
// Architecture_wrappers.py:197-267}.
#include "emt.h"

#include "gemm.h"

namespace tt2 {

// ---- reference encoder outputs ----------------------------------------------------------------
//
// TF1 GRUCell over every frame of the CNN output (dynamic_rnn / bidirectional_dynamic_rnn without
// sequence_length, so padded frames count, modules.py:38-53).  Block (b, g) runs GRU g of row b;
// xg [B][T2][NG][3D] holds x·[Wg_x | Wc_x] + [bg | bc] for every frame (one GEMM before).
//   mode 0 ('gru'): g = direction; g = 1 walks t = T2-1 .. 0 (the full-length reverse of
//                   bidirectional_dynamic_rnn) and writes its output back at t: out[b][t][g·D + i].
//   mode 1 ('gru_multi'): last output of GRU g -> dense(128, tanh): out[b][g][128].
__global__ __launch_bounds__(256) void k_emt_gru(const float* __restrict__ xg, int T2, int D, int NG,
                                                 const float* __restrict__ whg, const float* __restrict__ whc,
                                                 int mode, const float* __restrict__ kd,
                                                 const float* __restrict__ bd, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
  float* h = sm;          // [D]
  float* rh = h + D;      // [D]
  float* gates = rh + D;  // [2D] = [r | u]
  for (int i = tid; i < D; i += blockDim.x) h[i] = 0.f;
  __syncthreads();
  const float* Wg = whg + (long)g * D * 2 * D;
  const float* Wc = whc + (long)g * D * D;
  for (int s = 0; s < T2; ++s) {
    const int t = (mode == 0 && g == 1) ? T2 - 1 - s : s;
    const float* x = xg + ((long)b * T2 + t) * NG * 3 * D + (long)g * 3 * D;
    for (int j = tid; j < 2 * D; j += blockDim.x) {
      float acc = 0.f;
      for (int k = 0; k < D; ++k) acc = fmaf(h[k], Wg[(long)k * 2 * D + j], acc);
      gates[j] = sigm(x[j] + acc);
    }
    __syncthreads();
    for (int i = tid; i < D; i += blockDim.x) rh[i] = gates[i] * h[i];
    __syncthreads();
    float hn = 0.f;
    if (tid < D) {
      float acc = 0.f;
      for (int k = 0; k < D; ++k) acc = fmaf(rh[k], Wc[(long)k * D + tid], acc);
      const float cand = tanhf(x[2 * D + tid] + acc);
      const float u = gates[D + tid];
      hn = u * h[tid] + (1.f - u) * cand;
    }
    __syncthreads();
    if (tid < D) {
      h[tid] = hn;
      if (mode == 0) out[((long)b * T2 + t) * NG * D + (long)g * D + tid] = hn;
    }
    __syncthreads();
  }
  if (mode == 1 && tid < EMT_OUT) {
    const float* K = kd + (long)g * D * EMT_OUT;
    float acc = 0.f;
    for (int k = 0; k < D; ++k) acc = fmaf(h[k], K[(long)k * EMT_OUT + tid], acc);
    out[((long)b * NG + g) * EMT_OUT + tid] = tanhf(acc + bd[g * EMT_OUT + tid]);
  }
}

void gru_sequence(const float* xg, int B, int T, int D, int NG, const float* whg, const float* whc, int mode,
                  const float* kd, const float* bd, float* out, hipStream_t s) {
  TT2_CHECK(D >= 1 && D <= 256, TT2_ERR_INVALID_ARG, "gru_sequence: GRU units must be <= 256");
  hipLaunchKernelGGL(k_emt_gru, dim3(B, NG), dim3(256), sizeof(float) * 4 * D, s, xg, T, D, NG, whg, whc, mode, kd, bd,
                     out);
  TT2_HIP(hipGetLastError());
}

// style_tokens values: tanh(tokens) (tacotron_emt_attn.py:214; the batch tile is a broadcast)
__global__ void k_emt_tanh(const float* __restrict__ x, int n, float* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = tanhf(x[i]);
}

// per-row query bias: the query layer's bias, plus (style_tokens) the kernel row of the one-hot
// emotion label that concat([LSTM_output, labels]) multiplies (Architecture_wrappers.py:236);
// tf.one_hot of an out-of-range label is a zero row
__global__ void k_emt_qrow(const float* __restrict__ qb, const float* __restrict__ qlab,
                           const int* __restrict__ labels, int n_emt, int Aq, float* __restrict__ qrow) {
  const int b = blockIdx.x;
  for (int n = threadIdx.x; n < Aq; n += blockDim.x) {
    float v = qb[n];
    if (qlab) {
      const int l = labels[b];
      if (l >= 0 && l < n_emt) v += qlab[(long)l * Aq + n];
    }
    qrow[(long)b * Aq + n] = v;
  }
}

// ---- decoder step --------------------------------------------------------------------------------
// Σ_{k0 <= k < k1} x[k]·W[k·ld + col]: 8 independent accumulators so 8 weight loads are in flight
// per thread (one dependent chain of L2 loads would cost ~0.5 us per 2 k)
__device__ __forceinline__ float dot_col(const float* __restrict__ x, const float* __restrict__ W, int ld, int col, int k0,
                                         int k1) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = k0;
  for (; k + 8 <= k1; k += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = fmaf(x[k + u], W[(long)(k + u) * ld + col], acc[u]);
  }
  for (; k < k1; ++k) acc[0] = fmaf(x[k], W[(long)k * ld + col], acc[0]);
  return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

struct EmtStepArgs {
  const int* done;
  const float* Xp;                    // AF [32 x ...]: h2 = LSTM_output at columns [0, H)
  float* X1; int col0;                // AF next-step LSTM-1 input block
  const float* wq; const float* qrow; // [H][Aq], [B][Aq]
  const float* ke; long ke_bs;        // [Tv][Aq] per row
  const float* val; long val_bs;      // [Tv][Dv] per row
  const float* vv; const float* ab;   // [dh] score vector, [dh] pre-tanh bias (null: none)
  const float* wd; const float* bd;   // multi-head output dense [heads·Dv][128] (null: none)
  const float* spk; int spk_mode;     // [B][128]: 1 appended after the context, 2 added to it
  int H, Aq, heads, dh, Tv, Dv;
  float* hist;                        // [B][heads][Tv] of this step, or null
};

// One 512-thread block per batch row:
//   q = h2·Wq + qrow                                   (W2 / the multi-head query conv1d)
//   s[h][j] = Σ_d vv[d]·tanh(ke[j][h·dh+d] + q[h·dh+d] (+ ab[d]))
//           'simple': V(tanh(W1(values) + W2(query))) (attention.py:250; V's bias cancels in the
//           softmax); multi-head: normed_v = g·v/‖v‖ with attention_b (multihead_attention.py:97-115)
//   a = softmax_j s (no mask: the reference encoder's padded frames are attended too)
//   ctx[h] = Σ_j a[h][j]·values[j]; heads concatenated (_combine_heads)
//   'multihead': dense(128) (Architecture_wrappers.py:233-234), + refnet_spk (:206)
//   'simple': [ctx | refnet_spk] (:209); 'style_tokens': ctx (:211)
__global__ __launch_bounds__(512) void k_emt_step(EmtStepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (*a.done) return;
  const int b = blockIdx.x, tid = threadIdx.x;
  float* h2 = sm;                  // [H]
  float* part = h2 + a.H;          // [4][128]
  float* q = part + 4 * 128;       // [Aq]
  float* sc = q + a.Aq;            // [heads][Tv]
  float* comb = sc + a.heads * a.Tv;  // [heads·Dv]
  for (int k = tid; k < a.H; k += blockDim.x) h2[k] = a.Xp[af_idx(b, k)];
  __syncthreads();
  const int col = tid & 127, ks = tid >> 7;
  {
    float acc = 0.f;
    if (col < a.Aq) acc = dot_col(h2, a.wq, a.Aq, col, ks * a.H / 4, (ks + 1) * a.H / 4);
    part[ks * 128 + col] = acc;
  }
  __syncthreads();
  if (tid < a.Aq) q[tid] = ((part[tid] + part[128 + tid]) + (part[256 + tid] + part[384 + tid])) + a.qrow[(long)b * a.Aq + tid];
  __syncthreads();
  const float* ke = a.ke + b * a.ke_bs;
  const float* val = a.val + b * a.val_bs;
  for (int e = tid; e < a.heads * a.Tv; e += blockDim.x) {
    const int hh = e / a.Tv, j = e % a.Tv;
    float s = 0.f;
    for (int d = 0; d < a.dh; ++d) {
      float x = ke[(long)j * a.Aq + hh * a.dh + d] + q[hh * a.dh + d];
      if (a.ab) x += a.ab[d];
      s = fmaf(a.vv[d], tanhf(x), s);
    }
    sc[e] = s;
  }
  __syncthreads();
  if (tid < a.heads) {
    float* r = sc + tid * a.Tv;
    float mx = -INFINITY;
    for (int j = 0; j < a.Tv; ++j) mx = fmaxf(mx, r[j]);
    float sum = 0.f;
    for (int j = 0; j < a.Tv; ++j) {
      r[j] = expf(r[j] - mx);
      sum += r[j];
    }
    for (int j = 0; j < a.Tv; ++j) {
      r[j] = r[j] / sum;
      if (a.hist) a.hist[((long)b * a.heads + tid) * a.Tv + j] = r[j];
    }
  }
  __syncthreads();
  for (int e = tid; e < a.heads * a.Dv; e += blockDim.x) {
    const int hh = e / a.Dv, d = e % a.Dv;
    float s = 0.f;
    for (int j = 0; j < a.Tv; ++j) s = fmaf(sc[hh * a.Tv + j], val[(long)j * a.Dv + d], s);
    comb[e] = s;
  }
  __syncthreads();
  if (a.wd) {
    const int K = a.heads * a.Dv;
    part[ks * 128 + col] = dot_col(comb, a.wd, EMT_OUT, col, ks * K / 4, (ks + 1) * K / 4);
    __syncthreads();
    if (tid < EMT_OUT) {
      float o = ((part[tid] + part[128 + tid]) + (part[256 + tid] + part[384 + tid])) + a.bd[tid];
      if (a.spk_mode == 2) o += a.spk[(long)b * EMT_OUT + tid];
      a.X1[af_idx(b, a.col0 + tid)] = o;
    }
  } else {
    const int n = a.heads * a.Dv;
    for (int e = tid; e < n; e += blockDim.x) a.X1[af_idx(b, a.col0 + e)] = comb[e];
    if (a.spk_mode == 1 && tid < EMT_OUT) a.X1[af_idx(b, a.col0 + n + tid)] = a.spk[(long)b * EMT_OUT + tid];
  }
}

// zero_state: attention_emt = 0, so the block is [0 | spk] ('simple'), spk + 0 ('multihead') or 0
__global__ void k_emt_init(const float* __restrict__ spk, int spk_mode, int off, float* __restrict__ X1a,
                           float* __restrict__ X1b, int col0) {
  const int b = blockIdx.x, i = threadIdx.x;
  if (i >= EMT_OUT) return;
  const float v = spk[(long)b * EMT_OUT + i];
  const int k = af_idx(b, col0 + (spk_mode == 1 ? off : 0) + i);
  X1a[k] = v;
  X1b[k] = v;
}

// ---- host ------------------------------------------------------------------------------------------
static void up(DevBuf& d, const std::vector<float>& h) {
  d.alloc(h.size() * sizeof(float));
  TT2_HIP(hipMemcpy(d.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
}

void emt_configure(EmtModel& m, int attn, int ref_gru, int emt_only, int n_emt, int H, int attention_dim,
                   int style_att_dim, int num_heads, int ref_depth, int num_mels, const int filters[6],
                   int max_batch, int max_T_ref, int max_iters) {
  m.attn = attn;
  if (attn == EMT_OFF) return;
  TT2_CHECK(attn >= EMT_SIMPLE && attn <= EMT_STYLE_TOKENS, TT2_ERR_INVALID_ARG, "emt_attn must be 0..3");
  TT2_CHECK(ref_gru >= EMT_GRU_NONE && ref_gru <= EMT_GRU_MULTI, TT2_ERR_INVALID_ARG, "emt_ref_gru must be 0..2");
  m.ref_gru = ref_gru;
  m.spk = (attn != EMT_STYLE_TOKENS && !emt_only) ? 1 : 0;  // style_tokens builds no refnets (:209-216)
  m.n_emt = n_emt;
  m.H = H;
  m.D = ref_depth;
  m.max_batch = max_batch;
  m.max_iters = max_iters;
  int T2 = std::max(max_T_ref, 1), F = num_mels;
  for (int i = 0; i < 6; ++i) {
    T2 = (T2 + 1) / 2;
    F = (F + 1) / 2;
  }
  m.gin = F * filters[5];
  if (attn == EMT_STYLE_TOKENS) {
    TT2_CHECK(n_emt >= 1, TT2_ERR_INVALID_ARG, "style_tokens needs n_emt >= 1");
    m.Dv = EMT_TOKD;
    m.max_Tv = EMT_NTOK;
  } else {
    m.NG = ref_gru == EMT_GRU_BI ? 2 : ref_gru == EMT_GRU_MULTI ? EMT_NMULTI : 0;
    m.Dv = ref_gru == EMT_GRU_NONE ? m.gin : ref_gru == EMT_GRU_BI ? 2 * m.D : EMT_OUT;
    m.max_Tv = ref_gru == EMT_GRU_MULTI ? EMT_NMULTI : T2;
    TT2_CHECK(m.NG == 0 || m.D <= 256, TT2_ERR_INVALID_ARG, "reference_depth must be <= 256 for the emt GRUs");
  }
  if (attn == EMT_SIMPLE) {
    m.Aq = attention_dim;
    m.heads = 1;
    // the zero attention_emt state is attention_dim wide (Architecture_wrappers.py:116-117, 182);
    // a context of another width would change the LSTM input between steps: TF cannot build it
    TT2_CHECK(m.Dv == m.Aq, TT2_ERR_INVALID_ARG,
              "emt_attn 'simple': the reference-encoder output width (" + std::to_string(m.Dv) +
                  ") must equal attention_dim (" + std::to_string(m.Aq) + "); use emt_ref_gru 'gru_multi'");
    m.XW = m.Aq + (m.spk ? EMT_OUT : 0);
  } else {
    m.Aq = style_att_dim;
    m.heads = num_heads;
    TT2_CHECK(num_heads >= 1 && style_att_dim % num_heads == 0, TT2_ERR_INVALID_ARG,
              "style_att_dim must be a multiple of num_heads");
    if (attn == EMT_MULTIHEAD) {
      m.XW = EMT_OUT;  // dense(128); refnet_spk (128) is added, not concatenated
    } else {
      TT2_CHECK(num_heads * EMT_TOKD == 64, TT2_ERR_INVALID_ARG,
                "style_tokens: num_heads x 16 must be the 64-wide attention state (Architecture_wrappers.py:121)");
      m.XW = num_heads * EMT_TOKD;
    }
  }
  m.dh = m.Aq / m.heads;
  TT2_CHECK(m.Aq % 16 == 0 && m.Aq <= 128, TT2_ERR_INVALID_ARG, "emotion attention units must be a multiple of 16, <= 128");
  TT2_CHECK(m.heads * m.Dv <= 4096, TT2_ERR_INVALID_ARG, "emotion attention context too wide");
  m.qrow.alloc(sizeof(float) * 32 * m.Aq);
  m.labels.alloc(sizeof(int) * 32);
  TT2_HIP(hipMemset(m.labels.p, 0, m.labels.bytes));
  m.hist.alloc(sizeof(float) * (size_t)max_iters * max_batch * m.heads * m.max_Tv);
  if (m.attn != EMT_STYLE_TOKENS) {
    m.val.alloc(sizeof(float) * (size_t)max_batch * m.max_Tv * m.Dv);
    m.ke.alloc(sizeof(float) * (size_t)max_batch * m.max_Tv * m.Aq);
    if (m.NG) m.xg.alloc(sizeof(float) * (size_t)max_batch * T2 * m.NG * 3 * m.D);
  } else {
    m.val.alloc(sizeof(float) * EMT_NTOK * EMT_TOKD);
    m.ke.alloc(sizeof(float) * EMT_NTOK * m.Aq);
  }
}

void emt_load(EmtModel& m, const WeightMap& wm, const std::string& P) {
  if (!m.on()) return;
  const int H = m.H, Aq = m.Aq, D = m.D;
  if (m.NG) {
    // [gin][NG·3D] x rows of every GRU's gates | candidate kernels; recurrent rows per GRU
    std::vector<float> wx((size_t)m.gin * m.NG * 3 * D), bx((size_t)m.NG * 3 * D), whg, whc, kd, bd;
    for (int g = 0; g < m.NG; ++g) {
      const std::string s = m.ref_gru == EMT_GRU_BI
                                ? P + "refnet_emt/bidirectional_rnn/" + (g ? "bw" : "fw") + "/gru_cell/"
                                : P + "refnet_emt/gru_" + std::to_string(g) + "/rnn/gru_cell/";
      const auto& kg = need(wm, s + "gates/kernel", {m.gin + D, 2 * D});
      const auto& bg = need(wm, s + "gates/bias", {2 * D});
      const auto& kc = need(wm, s + "candidate/kernel", {m.gin + D, D});
      const auto& bc = need(wm, s + "candidate/bias", {D});
      const size_t ld = (size_t)m.NG * 3 * D, o = (size_t)g * 3 * D;
      for (int k = 0; k < m.gin; ++k) {
        for (int j = 0; j < 2 * D; ++j) wx[k * ld + o + j] = kg.data[(size_t)k * 2 * D + j];
        for (int j = 0; j < D; ++j) wx[k * ld + o + 2 * D + j] = kc.data[(size_t)k * D + j];
      }
      for (int j = 0; j < 2 * D; ++j) bx[o + j] = bg.data[j];
      for (int j = 0; j < D; ++j) bx[o + 2 * D + j] = bc.data[j];
      whg.insert(whg.end(), kg.data.begin() + (size_t)m.gin * 2 * D, kg.data.end());
      whc.insert(whc.end(), kc.data.begin() + (size_t)m.gin * D, kc.data.end());
      if (m.ref_gru == EMT_GRU_MULTI) {
        const std::string sd = P + "refnet_emt/gru_" + std::to_string(g) + "/dense/";
        const auto& k = need(wm, sd + "kernel", {D, EMT_OUT});
        const auto& b = need(wm, sd + "bias", {EMT_OUT});
        kd.insert(kd.end(), k.data.begin(), k.data.end());
        bd.insert(bd.end(), b.data.begin(), b.data.end());
      }
    }
    up(m.gwx, wx);
    up(m.gbx, bx);
    up(m.gwhg, whg);
    up(m.gwhc, whc);
    if (!kd.empty()) {
      up(m.gkd, kd);
      up(m.gbd, bd);
    }
  }
  if (m.attn == EMT_SIMPLE) {
    // Dense layers W1, W2, V built at their first call, inside the decoder cell (attention.py:237-250)
    up(m.wk, need(wm, P + "decoder/W1/kernel", {m.Dv, Aq}).data);
    up(m.bk, need(wm, P + "decoder/W1/bias", {Aq}).data);
    up(m.wq, need(wm, P + "decoder/W2/kernel", {H, Aq}).data);
    up(m.qb, need(wm, P + "decoder/W2/bias", {Aq}).data);
    up(m.vv, need(wm, P + "decoder/V/kernel", {Aq, 1}).data);
    (void)need(wm, P + "decoder/V/bias", {1});  // shifts every score equally: no effect on the softmax
    m.ab.free();
  } else {
    const std::string mh = P + "decoder/Multihead-attention-attn_emt/";
    const int Kq = H + (m.attn == EMT_STYLE_TOKENS ? m.n_emt : 0);
    const auto& kq = need(wm, mh + "conv1d/kernel", {1, Kq, Aq});
    up(m.wq, std::vector<float>(kq.data.begin(), kq.data.begin() + (size_t)H * Aq));
    if (m.attn == EMT_STYLE_TOKENS)
      up(m.qlab, std::vector<float>(kq.data.begin() + (size_t)H * Aq, kq.data.end()));
    up(m.qb, need(wm, mh + "conv1d/bias", {Aq}).data);
    up(m.wk, need(wm, mh + "conv1d_1/kernel", {1, m.Dv, Aq}).data);
    up(m.bk, need(wm, mh + "conv1d_1/bias", {Aq}).data);
    // normed_v = g·v·rsqrt(Σ v²) (multihead_attention.py:108-110), folded once
    const auto& v = need(wm, mh + "attention_v", {m.dh});
    const float g = need(wm, mh + "attention_g", {}).data[0];
    float ss = 0.f;
    for (float x : v.data) ss += x * x;
    const float r = 1.0f / sqrtf(ss);
    std::vector<float> nv(m.dh);
    for (int d = 0; d < m.dh; ++d) nv[d] = g * v.data[d] * r;
    up(m.vv, nv);
    up(m.ab, need(wm, mh + "attention_b", {m.dh}).data);
    if (m.attn == EMT_MULTIHEAD) {
      up(m.wd, need(wm, P + "decoder/attn_emt/dense/kernel", {m.heads * m.Dv, EMT_OUT}).data);
      up(m.bd, need(wm, P + "decoder/attn_emt/dense/bias", {EMT_OUT}).data);
    } else {
      up(m.tokens, need(wm, P + "style_tokens", {EMT_NTOK, EMT_TOKD}).data);
    }
  }
}

void emt_encode(EmtModel& m, const float* x, int B, int T2, hipStream_t s) {
  if (!m.on()) return;
  m.B = B;
  const float* vals = nullptr;
  int rows = 0;
  if (m.attn == EMT_STYLE_TOKENS) {
    m.Tv = EMT_NTOK;
    hipLaunchKernelGGL(k_emt_tanh, dim3(cdiv(EMT_NTOK * EMT_TOKD, 256)), dim3(256), 0, s, m.tokens.as<float>(),
                       EMT_NTOK * EMT_TOKD, m.val.as<float>());
    vals = m.val.as<float>();
    rows = EMT_NTOK;
  } else {
    TT2_CHECK(x, TT2_ERR_INVALID_ARG, "emt_encode: reference CNN output missing");
    m.Tv = m.ref_gru == EMT_GRU_MULTI ? EMT_NMULTI : T2;
    TT2_CHECK(m.Tv <= m.max_Tv, TT2_ERR_SHAPE_MISMATCH, "emotion reference exceeds max_T_ref");
    if (m.ref_gru == EMT_GRU_NONE) {
      // ReferenceEncoder all_outputs without a GRU: the reshaped CNN output itself (modules.py:31-55)
      TT2_HIP(hipMemcpyAsync(m.val.p, x, sizeof(float) * (size_t)B * T2 * m.gin, hipMemcpyDeviceToDevice, s));
    } else {
      GemmArgs g;
      g.M = B * T2; g.N = m.NG * 3 * m.D; g.K = m.gin; g.A = x; g.lda = m.gin;
      g.Bw = m.gwx.as<float>(); g.ldb = g.N; g.Cout = m.xg.as<float>(); g.ldc = g.N; g.bias = m.gbx.as<float>();
      gemm(g, s);
      gru_sequence(m.xg.as<float>(), B, T2, m.D, m.NG, m.gwhg.as<float>(), m.gwhc.as<float>(),
                   m.ref_gru == EMT_GRU_MULTI ? 1 : 0, m.gkd.as<float>(), m.gbd.as<float>(), m.val.as<float>(), s);
    }
    vals = m.val.as<float>();
    rows = B * m.Tv;
  }
  {  // keys: W1(values) ('simple') / conv1d(value) (multi-head), for every value row at once
    GemmArgs g;
    g.M = rows; g.N = m.Aq; g.K = m.Dv; g.A = vals; g.lda = m.Dv;
    g.Bw = m.wk.as<float>(); g.ldb = m.Aq; g.Cout = m.ke.as<float>(); g.ldc = m.Aq; g.bias = m.bk.as<float>();
    gemm(g, s);
  }
  hipLaunchKernelGGL(k_emt_qrow, dim3(B), dim3(128), 0, s, m.qb.as<float>(),
                     m.attn == EMT_STYLE_TOKENS ? m.qlab.as<float>() : nullptr, m.labels.as<int>(), m.n_emt, m.Aq,
                     m.qrow.as<float>());
  TT2_HIP(hipGetLastError());
}

void emt_init_launch(const EmtModel& m, const float* spk, float* X1a, float* X1b, int col0, hipStream_t s) {
  if (!m.on() || !m.spk) return;
  const int mode = m.attn == EMT_SIMPLE ? 1 : 2;
  hipLaunchKernelGGL(k_emt_init, dim3(m.B), dim3(EMT_OUT), 0, s, spk, mode, m.heads * m.Dv, X1a, X1b, col0);
  TT2_HIP(hipGetLastError());
}

void emt_step_launch(const EmtModel& m, const int* done, const float* Xp, float* X1, int col0, const float* spk, int t,
                     hipStream_t s) {
  EmtStepArgs a;
  a.done = done; a.Xp = Xp; a.X1 = X1; a.col0 = col0;
  a.wq = m.wq.as<float>(); a.qrow = m.qrow.as<float>();
  a.ke = m.ke.as<float>(); a.ke_bs = m.ke_bstride();
  a.val = m.val.as<float>(); a.val_bs = m.val_bstride();
  a.vv = m.vv.as<float>(); a.ab = m.ab.p ? m.ab.as<float>() : nullptr;
  a.wd = m.attn == EMT_MULTIHEAD ? m.wd.as<float>() : nullptr;
  a.bd = m.attn == EMT_MULTIHEAD ? m.bd.as<float>() : nullptr;
  a.spk = spk;
  a.spk_mode = !m.spk ? 0 : m.attn == EMT_SIMPLE ? 1 : 2;
  a.H = m.H; a.Aq = m.Aq; a.heads = m.heads; a.dh = m.dh; a.Tv = m.Tv; a.Dv = m.Dv;
  a.hist = t < m.max_iters ? m.hist.as<float>() + (size_t)t * m.B * m.heads * m.Tv : nullptr;
  const size_t shm = sizeof(float) * (m.H + 4 * 128 + m.Aq + m.heads * m.Tv + m.heads * m.Dv);
  hipLaunchKernelGGL(k_emt_step, dim3(m.B), dim3(512), shm, s, a);
}

}  // namespace tt2
