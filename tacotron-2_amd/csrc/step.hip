// tt2_decoder_step kernels (step.h): one TacotronDecoderCell.__call__ (Architecture_wrappers.py:
// 197-267) from an explicit state, in plain fp32 (every dot product one thread, k in order).
#include "step.h"

namespace tt2 {

enum StepAct { SA_NONE = 0, SA_PRENET = 1, SA_SIGMOID = 2 };

// out[b][n] = act(cat(x0[b][:k0], x1[b][:k1], x2[b][:k2]) · W[:, n] + bias[n])
//   SA_PRENET: Prenet layer (modules.py:352-356): dropout(relu(y), 0.5, training=True) =
//              relu(y) / 0.5 · keep (tf.layers.dropout); SA_SIGMOID: StopProjection at inference
//              (modules.py:446-448).
__global__ void k_step_dense(const float* __restrict__ x0, int k0, const float* __restrict__ x1, int k1,
                             const float* __restrict__ x2, int k2, const float* __restrict__ W,
                             const float* __restrict__ bias, int N, float* __restrict__ out, int act,
                             const uint8_t* __restrict__ keep) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
  if (n >= N) return;
  float acc = 0.f;
  const float* xs[3] = {x0, x1, x2};
  const int ks[3] = {k0, k1, k2};
  int row = 0;
  for (int seg = 0; seg < 3; ++seg) {
    const float* x = xs[seg] + (long)b * ks[seg];
    for (int k = 0; k < ks[seg]; ++k) acc = fmaf(x[k], W[(long)(row + k) * N + n], acc);
    row += ks[seg];
  }
  float y = acc + (bias ? bias[n] : 0.f);
  if (act == SA_PRENET) y = (fmaxf(y, 0.f) / 0.5f) * (float)keep[(long)b * N + n];
  else if (act == SA_SIGMOID) y = 1.f / (1.f + expf(-y));
  out[(long)b * N + n] = y;
}

// TF1 LSTMCell update (gates [i, j, f, o], forget_bias 1) + inference zoneout (modules.py:220-248):
// h_new = the emitted (un-zoned) output, (c_out, h_out) = the carried zoneout mix.
__global__ void k_step_cell(const float* __restrict__ z, const float* __restrict__ c_prev,
                            const float* __restrict__ h_prev, int B, int H, float zo, float* __restrict__ h_new,
                            float* __restrict__ c_out, float* __restrict__ h_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H) return;
  const int b = i / H, u = i % H;
  const float* g = z + (long)b * 4 * H;
  const float zi = g[u], zj = g[H + u], zf = g[2 * H + u], zz = g[3 * H + u];
  const float cp = c_prev[i], hp = h_prev[i];
  const float cn = sigm(zf + 1.0f) * cp + sigm(zi) * tanhf(zj);
  const float hn = sigm(zz) * tanhf(cn);
  h_new[i] = hn;
  c_out[i] = (1.f - zo) * cn + zo * cp;
  h_out[i] = (1.f - zo) * hn + zo * hp;
}

// Location-sensitive energies (attention.py:37-69, 186-201): f = conv1d_same(cum, W_conv) (its bias
// is folded into keys), loc = f·W_loc, e_j = Σ_k v_a[k]·tanh(keys_jk + q_k + loc_jk) -- keys carry
// b_a + b_conv·W_loc.  One thread per (b, j).
__global__ void k_step_energy(const float* __restrict__ keys, const float* __restrict__ q,
                              const float* __restrict__ cum, const float* __restrict__ wconv,
                              const float* __restrict__ wloc, const float* __restrict__ va, int B, int T, int A,
                              int F, int KL, float* __restrict__ energy) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
  if (j >= T) return;
  const int pl = (KL - 1) / 2;
  float f[32];
  for (int ff = 0; ff < F; ++ff) {
    float s = 0.f;
    for (int tap = 0; tap < KL; ++tap) {
      const int src = j + tap - pl;
      if (src >= 0 && src < T) s = fmaf(cum[(long)b * T + src], wconv[tap * F + ff], s);
    }
    f[ff] = s;
  }
  float e = 0.f;
  for (int k = 0; k < A; ++k) {
    float loc = 0.f;
    for (int ff = 0; ff < F; ++ff) loc = fmaf(f[ff], wloc[ff * A + k], loc);
    e = fmaf(va[k], tanhf(keys[((long)b * T + j) * A + k] + q[(long)b * A + k] + loc), e);
  }
  energy[(long)b * T + j] = e;
}

// Synthesis window / monotonic constraint (attention.py:202-215), memory mask (TF
// _maybe_mask_score), softmax (:218), max_attentions = argmax (:219), cumulative state (:222-225).
// One 256-thread block per row.
__global__ void k_step_softmax(const float* __restrict__ energy, const float* __restrict__ cum,
                               const int* __restrict__ max_att, const int* __restrict__ lengths, int T,
                               int constraint, int monotonic, int win, int mask_encoder, int cumulative,
                               int smoothing, float* __restrict__ align, float* __restrict__ cum_out, int* __restrict__ max_att_o) {
  __shared__ float red[256];
  __shared__ int redi[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int len = lengths[b], pm = max_att[b];
  auto score = [&](int j) {
    float e = energy[(long)b * T + j];
    if (constraint) {
      const bool masked = monotonic ? (j < pm || j >= pm + win)
                                    : (j < pm - (win / 2 + (win % 2 != 0 ? 1 : 0)) || j >= pm + win / 2);
      if (masked) e = -4294967296.0f;  // -2**32 + 1 in fp32
    }
    if (mask_encoder && j >= len) e = -INFINITY;
    return e;
  };
  // probability_fn: softmax, or _smoothing_normalization (attention.py:71-80) = sigmoid / sum sigmoid
  auto prob = [&](int j, float mx) { return smoothing ? 1.f / (1.f + expf(-score(j))) : expf(score(j) - mx); };
  float mx = -INFINITY;
  for (int j = tid; j < T; j += blockDim.x) mx = fmaxf(mx, score(j));
  red[tid] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmaxf(red[tid], red[tid + o]);
    __syncthreads();
  }
  mx = red[0];
  __syncthreads();
  float sum = 0.f;
  for (int j = tid; j < T; j += blockDim.x) sum += prob(j, mx);
  red[tid] = sum;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  sum = red[0];
  __syncthreads();
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = tid; j < T; j += blockDim.x) {
    const float a = prob(j, mx) / sum;
    align[(long)b * T + j] = a;
    cum_out[(long)b * T + j] = cumulative ? a + cum[(long)b * T + j] : a;
    if (a > best) {
      best = a;
      bi = j;
    }
  }
  red[tid] = best;
  redi[tid] = bi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const float ob = red[tid + o];
      const int oi = redi[tid + o];
      if (ob > red[tid] || (ob == red[tid] && oi < redi[tid])) {
        red[tid] = ob;
        redi[tid] = oi;
      }
    }
    __syncthreads();
  }
  if (tid == 0) max_att_o[b] = redi[0];
}

// context = alignments · values (attention.py:27)
__global__ void k_step_context(const float* __restrict__ align, const float* __restrict__ values, int T, int D,
                               float* __restrict__ ctx) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
  if (d >= D) return;
  float s = 0.f;
  for (int j = 0; j < T; ++j) s = fmaf(align[(long)b * T + j], values[((long)b * T + j) * D + d], s);
  ctx[(long)b * D + d] = s;
}

size_t step_scratch_floats(const StepDims& d) {
  return (size_t)d.B * (2 * d.P + 4 * d.H + 2 * d.H + d.A + d.T);
}

void decoder_step_launch(const StepWeights& w, const StepDims& d, const StepIO& io, hipStream_t s) {
  TT2_CHECK(d.F <= 32, TT2_ERR_INVALID_ARG, "tt2_decoder_step: attention_filters > 32");
  const int B = d.B;
  float* x1 = io.scratch;              // [B][P] prenet layer 1
  float* x2 = x1 + (size_t)B * d.P;    // [B][P] prenet output
  float* z = x2 + (size_t)B * d.P;     // [B][4H] gate pre-activations
  float* o1 = z + (size_t)B * 4 * d.H; // [B][H] layer-1 emitted output
  float* o2 = o1 + (size_t)B * d.H;    // [B][H] layer-2 emitted output
  float* q = o2 + (size_t)B * d.H;     // [B][A] query
  float* en = q + (size_t)B * d.A;     // [B][T] energies
  auto dense = [&](const float* a0, int k0, const float* a1, int k1, const float* a2, int k2, const float* W,
                   const float* bias, int N, float* out, int act, const uint8_t* keep) {
    hipLaunchKernelGGL(k_step_dense, dim3(cdiv(N, 256), B), dim3(256), 0, s, a0, k0, a1, k1, a2, k2, W, bias, N,
                       out, act, keep);
  };
  // Prenet (modules.py:346-357) on the previous frame (TacoTestHelper feeds it raw, helpers.py:57)
  dense(io.frame_in, d.nm, nullptr, 0, nullptr, 0, w.pre_w1, w.pre_b1, d.P, x1, SA_PRENET, io.masks);
  dense(x1, d.P, nullptr, 0, nullptr, 0, w.pre_w2, w.pre_b2, d.P, x2, SA_PRENET, io.masks + (size_t)B * d.P);
  // DecoderRNN (modules.py:360-389): layer 1 on [prenet, context] (Architecture_wrappers.py:202-214)
  dense(x2, d.P, io.ctx, d.D, io.h1, d.H, w.k1, w.b1, 4 * d.H, z, SA_NONE, nullptr);
  const int nbh = cdiv(B * d.H, 256);
  hipLaunchKernelGGL(k_step_cell, dim3(nbh), dim3(256), 0, s, z, io.c1, io.h1, B, d.H, d.zo, o1, io.c1o, io.h1o);
  dense(o1, d.H, io.h2, d.H, nullptr, 0, w.k2, w.b2, 4 * d.H, z, SA_NONE, nullptr);
  hipLaunchKernelGGL(k_step_cell, dim3(nbh), dim3(256), 0, s, z, io.c2, io.h2, B, d.H, d.zo, o2, io.c2o, io.h2o);
  // LocationSensitiveAttention (attention.py:170-227) on the layer-2 output
  dense(o2, d.H, nullptr, 0, nullptr, 0, w.wq, nullptr, d.A, q, SA_NONE, nullptr);
  hipLaunchKernelGGL(k_step_energy, dim3(cdiv(d.T, 64), B), dim3(64), 0, s, io.keys, q, io.cum, w.wconv, w.wloc, w.va,
                     B, d.T, d.A, d.F, d.KL, en);
  hipLaunchKernelGGL(k_step_softmax, dim3(B), dim3(256), 0, s, en, io.cum, io.max_att, io.lengths, d.T, d.constraint,
                     d.monotonic, d.win, d.mask_encoder, d.cumulative, d.smoothing, io.align, io.cumo, io.max_att_o);
  hipLaunchKernelGGL(k_step_context, dim3(cdiv(d.D, 256), B), dim3(256), 0, s, io.align, io.values, d.T, d.D,
                     io.ctxo);
  // FrameProjection / StopProjection on [h2_new, context] (Architecture_wrappers.py:243-247)
  dense(o2, d.H, io.ctxo, d.D, nullptr, 0, w.wf, w.bf, d.nm, io.frame, SA_NONE, nullptr);
  dense(o2, d.H, io.ctxo, d.D, nullptr, 0, w.ws, w.bs, 1, io.stop, SA_SIGMOID, nullptr);
  TT2_HIP(hipGetLastError());
}

}  // namespace tt2
