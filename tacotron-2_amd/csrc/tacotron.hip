// Tacotron-2 synthesis path on MI355X (gfx950): encoder, reference encoders + GST, attention
// memory, the autoregressive decoder (prenet → 2×Zoneout-LSTM → location-sensitive attention →
// frame/stop projection) and the Postnet.  See DESIGN.md for the data layout and roofline.
//
// Reference: code/tacotron/models/{tacotron.py, modules.py, attention.py,
// Architecture_wrappers.py, helpers.py, custom_decoder.py, multihead_attention.py}.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <tuple>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <mutex>
#include <set>
#include "common.h"
#include "decode_persist.h"
#include "gemm.h"
#include "cbhg.h"
#include "emt.h"
#include "step.h"

namespace tt2 {

static thread_local std::string g_last_error;
void set_last_error(const std::string& m) { g_last_error = m; }

// TT2_SEGV_TRACE=1 (debug): a SIGSEGV / SIGABRT prints the native backtrace to stderr before the
// default action (the rocprofv3 exit crash of round 2 left only "Segmentation fault")
static void tt2_fatal_signal(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char* m = sig == SIGSEGV ? "libtt2: SIGSEGV, native backtrace:\n" : "libtt2: fatal signal, native backtrace:\n";
  (void)!write(2, m, strlen(m));
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
static const bool g_segv_trace = [] {
  const char* e = std::getenv("TT2_SEGV_TRACE");
  if (!e || !e[0] || e[0] == '0') return false;
  signal(SIGSEGV, tt2_fatal_signal);
  signal(SIGABRT, tt2_fatal_signal);
  return true;
}();

// TT2_REDZONE debug registry (common.h): every live DevBuf with a redzone
static std::mutex& rz_mu() {
  static std::mutex m;
  return m;
}
static std::set<DevBuf*>& rz_set() {
  static std::set<DevBuf*> s;
  return s;
}
void redzone_register(DevBuf* b, bool add) {
  std::lock_guard<std::mutex> l(rz_mu());
  if (add) rz_set().insert(b);
  else rz_set().erase(b);
}
std::string redzone_check_all(const char* phase) { return redzone_check(phase, nullptr, nullptr); }
std::string redzone_check(const char* phase, std::string (*namer)(const void*, const DevBuf*), const void* owner) {
  if (!redzone_on()) return "";
  TT2_HIP(hipDeviceSynchronize());
  std::lock_guard<std::mutex> l(rz_mu());
  std::vector<unsigned char> h(kRedzone);
  std::string out;
  for (DevBuf* b : rz_set()) {
    TT2_HIP(hipMemcpy(h.data(), static_cast<char*>(b->p) + b->bytes, kRedzone, hipMemcpyDeviceToHost));
    size_t first = kRedzone, last = 0;
    for (size_t i = 0; i < kRedzone; ++i)
      if (h[i] != kRedByte) {
        first = std::min(first, i);
        last = i;
      }
    if (first == kRedzone) continue;
    // re-arm, so a later call reports its own overflows rather than this one again
    TT2_HIP(hipMemset(static_cast<char*>(b->p) + b->bytes, kRedByte, kRedzone));
    TT2_HIP(hipDeviceSynchronize());
    std::string name = namer ? namer(owner, b) : std::string();
    if (name.empty()) name = "?";
    out += std::string("[") + phase + "] redzone of " + name + " (" + std::to_string(b->bytes) +
           " bytes) written at +" + std::to_string(first) + "..+" + std::to_string(last) + "; ";
  }
  return out;
}

void put_tensor(WeightMap& wm, const char* name, const float* host, const int64_t* shape, int ndim) {
  TT2_CHECK(name && host && ndim >= 0 && (ndim == 0 || shape), TT2_ERR_INVALID_ARG,
            "load_tensor: null argument");
  HostTensor t;
  int64_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    TT2_CHECK(shape[i] >= 0, TT2_ERR_INVALID_ARG, "load_tensor: negative dim");
    t.shape.push_back(shape[i]);
    n *= shape[i];
  }
  t.data.assign(host, host + n);
  wm[name] = std::move(t);
}

const HostTensor& need(const WeightMap& wm, const std::string& name, std::vector<int64_t> shape) {
  auto it = wm.find(name);
  TT2_CHECK(it != wm.end(), TT2_ERR_NOT_LOADED, "missing weight: " + name);
  std::vector<int64_t> got = it->second.shape;
  // scalars may come as () or (1,)
  auto squeeze = [](std::vector<int64_t> v) {
    std::vector<int64_t> r;
    for (auto d : v)
      if (d != 1) r.push_back(d);
    return r;
  };
  if (squeeze(got) != squeeze(shape)) {
    std::string s = "shape mismatch for " + name + ": got (";
    for (auto d : got) s += std::to_string(d) + ",";
    s += ") want (";
    for (auto d : shape) s += std::to_string(d) + ",";
    throw Error(TT2_ERR_SHAPE_MISMATCH, s + ")");
  }
  return it->second;
}

static const char* TP = "Tacotron_model/inference/";

// ==========================================================================================
// Device kernels
// ==========================================================================================

// ---- encoder -----------------------------------------------------------------------------

// embedding_lookup (tacotron.py:215-217): x[b,t,:] = table[ids[b,t], :]
__global__ void k_embed(const int* __restrict__ ids, const float* __restrict__ table, float* __restrict__ x,
                        int BT, int E, int n_sym) {
  const int row = blockIdx.x;
  if (row >= BT) return;
  int id = ids[row];
  id = id < 0 ? 0 : (id >= n_sym ? n_sym - 1 : id);
  for (int e = threadIdx.x; e < E; e += blockDim.x) x[(long)row * E + e] = table[(long)id * E + e];
}

// One time step of both directions of the encoder Zoneout-BiLSTM (modules.py:313-323) with
// tf.nn.bidirectional_dynamic_rnn sequence_length semantics.  Block = (dir, 4 hidden units).
// gates = xproj[b, pos, dir] (x·Wx + b, precomputed for every t by one GEMM) + h_prev·Wh.
struct EncLstmArgs {
  const float* xproj;   // [B*T][2*4U]
  const float* wh;      // [2][U/4][U x 16 WF tile]
  float* hs;            // [2 dirs][2 parity][32 x U AF]
  float* cs;            // [2][32][U]
  float* out;           // [B][T][2U]
  const int* lengths;
  int B, T, U, t;
  float zo, one_m_zo;
};

__global__ __launch_bounds__(256) void k_enc_lstm_step(EncLstmArgs a) {
  __shared__ float red[4 * 512];
  __shared__ float G[512];
  const int ng = a.U / 4;
  const int dir = blockIdx.x / ng, g = blockIdx.x % ng;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int par = a.t & 1;
  const float* X = a.hs + ((long)(dir * 2 + par) * 32 * a.U);
  float* Xn = a.hs + ((long)(dir * 2 + (par ^ 1)) * 32 * a.U);
  const float* Wt = a.wh + ((long)(dir * ng + g) * a.U * 16);
  const int nsg = a.U / 16;
  const int sg0 = wave * nsg / 4, sg1 = (wave + 1) * nsg / 4;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  skinny_mfma(X, Wt, sg0, sg1, acc0, acc1, lane);
  reduce_waves_32x16<4>(acc0, acc1, red, G, wave, lane, tid);
  if (tid < 128) {
    const int m = tid >> 2, uu = tid & 3, u = 4 * g + uu;
    const int U = a.U;
    const float hprev = X[af_idx(m, u)];
    float* cp = a.cs + ((long)dir * 32 + m) * U + u;
    bool act = false;
    int pos = 0;
    if (m < a.B) {
      const int L = a.lengths[m];
      act = a.t < L;
      pos = dir == 0 ? a.t : L - 1 - a.t;
    }
    if (act) {
      const float* xp = a.xproj + ((long)m * a.T + pos) * (8 * U) + dir * 4 * U;
      const float zi = G[m * 16 + 0 * 4 + uu] + xp[0 * U + u];
      const float zj = G[m * 16 + 1 * 4 + uu] + xp[1 * U + u];
      const float zf = G[m * 16 + 2 * 4 + uu] + xp[2 * U + u];
      const float zz = G[m * 16 + 3 * 4 + uu] + xp[3 * U + u];
      const float cprev = *cp;
      const float cn = sigm(zf + 1.0f) * cprev + sigm(zi) * tanhf(zj);
      const float hn = sigm(zz) * tanhf(cn);
      *cp = a.one_m_zo * cn + a.zo * cprev;
      Xn[af_idx(m, u)] = a.one_m_zo * hn + a.zo * hprev;
      a.out[((long)m * a.T + pos) * (2 * U) + dir * U + u] = hn;
    } else {
      Xn[af_idx(m, u)] = hprev;  // state copied through past the row's length
    }
  }
}

// Persistent BiLSTM (fork-default U = 256): the whole recurrence as ONE launch of 2 x U/4
// work-groups, work-group (dir, g) owning units [4g, 4g+4) of one direction with its recurrent
// weight tile in registers.  h of step t travels to the direction's U/4 work-groups as AF-ordered
// data-tagged 8-byte granules {tag = t+1, zoned h} (the data is the flag: one round trip per step,
// cdna_hip_programming.md §6 Guideline 16 R2); every spin is bounded.  Same arithmetic as
// k_enc_lstm_step.
typedef __attribute__((address_space(1))) unsigned long long enc_gu64;
typedef __attribute__((address_space(1))) int enc_gi32;
constexpr int ENC_U = 256;
struct EncPArgs {
  const float* xproj;  // [B][T][8U]: x·W_x + b for both directions
  const float* wh;     // [2][U/4 tiles][U x 16] WF
  unsigned long long* Hg;  // [2 dirs][2 parities][32 x U] AF granules (zeroed before the launch)
  float* out;          // [B][T][2U]
  const int* lengths;
  int B, T, Tmax;
  float zo, one_m_zo;
  int* err;            // timeout flag
  int sentinel;        // poll one sentinel granule per producer before the full h load (TT2_ENC_SENTINEL)
};

__global__ __launch_bounds__(256) void k_enc_bilstm_persist(EncPArgs a) {
  __shared__ float red[4 * 512];
  __shared__ float G[512];
  constexpr int U = ENC_U, ng = U / 4, NKG = U / 64;  // k-groups per wave
  const int dir = blockIdx.x / ng, g = blockIdx.x % ng;
  const int tid0 = threadIdx.x;
  f32x4 wt[NKG];
  {
    const f32x4* Wt = reinterpret_cast<const f32x4*>(a.wh + ((long)(dir * ng + g) * U * 16));
    const int w = tid0 >> 6, lane = tid0 & 63;
#pragma unroll
    for (int i = 0; i < NKG; ++i) wt[i] = Wt[(NKG * w + i) * 64 + lane] * KG_SB;  // pre-scaled (common.h)
  }
  const int m = (tid0 >> 2) & 31, uu = tid0 & 3, u = 4 * g + uu;
  const int L = (tid0 < 128 && m < a.B) ? a.lengths[m] : 0;
  float c = 0.f, hz = 0.f;  // cell and zoned hidden state of (m, u), threads < 128
  unsigned long long* const Hd = a.Hg + (long)dir * 2 * 32 * U;
  const auto r0 = __builtin_amdgcn_make_buffer_rsrc(Hd, (short)0, 0x7fffffff, 0x00020000);
  const auto r1 = __builtin_amdgcn_make_buffer_rsrc(Hd + 32 * U, (short)0, 0x7fffffff, 0x00020000);
  for (int t = 0; t < a.Tmax; ++t) {
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, w = tid >> 6;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    // this step's input projections, loaded before the h hand-off (off the serial chain)
    const bool act = tid < 128 && t < L;
    float xz[4] = {0.f, 0.f, 0.f, 0.f};
    const int pos = dir == 0 ? t : L - 1 - t;
    if (act) {
      const float* xp = a.xproj + ((long)m * a.T + pos) * (8 * U) + dir * 4 * U;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) xz[gq] = xp[gq * U + u];
    }
    if (t > 0) {  // h(t-1): parity (t-1)&1, tag t
      const auto rp = (t & 1) ? r0 : r1;
      f32x4 x0[NKG], x1[NKG];
      long long t0 = 0;
      // cheap poll first: one sentinel granule (row 0 of the producer's first unit) per producer
      // work-group of this wave's k-slice (units [U/4·w, U/4·(w+1)) = producers [16w, 16w+16))
      for (unsigned spin = 0; a.sentinel; ++spin) {
        bool ok = true;
        if (lane < U / 16) {
          const unsigned long long* sp = Hd + ((t - 1) & 1) * 32 * U + af_idx(0, 4 * (U / 16 * w + lane));
          ok = (unsigned)(__hip_atomic_load((enc_gu64*)sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) ==
               (unsigned)t;
        }
        if (__all(ok)) break;
        if ((spin & 31) == 0) {
          const long long now = __builtin_amdgcn_s_memrealtime();
          if (spin == 0) {
            t0 = now;
          } else if (__hip_atomic_load((enc_gi32*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                     now - t0 > 200000000LL) {
            if (lane == 0) __hip_atomic_store((enc_gi32*)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
      for (unsigned spin = 0;; ++spin) {  // then every granule, verified (rarely re-read)
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NKG; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int fo = (((NKG * w + i) * 2 + h) * 64 + lane) * 4;
            const auto q0 = __builtin_amdgcn_raw_buffer_load_b128(rp, fo * 8, 0, 16);
            const auto q1 = __builtin_amdgcn_raw_buffer_load_b128(rp, fo * 8 + 16, 0, 16);
            const f32x4 v = {__uint_as_float(q0[0]), __uint_as_float(q0[2]), __uint_as_float(q1[0]),
                             __uint_as_float(q1[2])};
            ok = ok && q0[1] == (unsigned)t && q0[3] == (unsigned)t && q1[1] == (unsigned)t && q1[3] == (unsigned)t;
            if (h == 0) x0[i] = v;
            else x1[i] = v;
          }
        if (__all(ok)) break;
        if ((spin & 31) == 0) {
          const long long now = __builtin_amdgcn_s_memrealtime();
          if (spin == 0) {
            t0 = now;
          } else if (__hip_atomic_load((enc_gi32*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                     now - t0 > 200000000LL) {
            if (lane == 0) __hip_atomic_store((enc_gi32*)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;  // whole wave; the others time out or see err the same way
          }
        }
        __builtin_amdgcn_s_sleep(2);
      }
#pragma unroll
      for (int i = 0; i < NKG; ++i) kg_mfma_x3(x0[i], x1[i], wt[i], acc0, acc1);  // split fp16x3 (common.h)
    }
    reduce_waves_32x16<4>(acc0, acc1, red, G, w, lane, tid);
    if (tid < 128) {
      if (act) {
        const float zi = G[m * 16 + 0 * 4 + uu] * KG_UNSCALE + xz[0];
        const float zj = G[m * 16 + 1 * 4 + uu] * KG_UNSCALE + xz[1];
        const float zf = G[m * 16 + 2 * 4 + uu] * KG_UNSCALE + xz[2];
        const float zz = G[m * 16 + 3 * 4 + uu] * KG_UNSCALE + xz[3];
        const float cn = sigm(zf + 1.0f) * c + sigm(zi) * tanhf(zj);
        const float hn = sigm(zz) * tanhf(cn);
        c = a.one_m_zo * cn + a.zo * c;
        hz = a.one_m_zo * hn + a.zo * hz;
        a.out[((long)m * a.T + pos) * (2 * U) + dir * U + u] = hn;
      }  // past the row's length the state is carried through unchanged
      __hip_atomic_store((enc_gu64*)(Hd + (t & 1) * 32 * U + af_idx(m, u)),
                         ((unsigned long long)(t + 1) << 32) | __float_as_uint(hz), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ReferenceEncoder GRU + dense(tanh) (modules.py:57-64) and GST MultiheadAttention
// (multihead_attention.py:35-132, tacotron.py:276-282) for one batch row.
struct RefGstArgs {
  const float* xg;       // [B][T2][3D]: x_t·[Wg_x | Wc_x] + [bg | bc] for every frame (one GEMM)
  int T2, D;             // D = reference_depth (GRU units)
  const float* whg;      // [D][2D] recurrent rows of the gates kernel
  const float* whc;      // [D][D]  recurrent rows of the candidate kernel
  const float* kd; const float* bd;  // [D][128], [128]
  const float* tokens;               // [ntok][tokd]
  const float* kq; const float* bq;  // [128][A], [A]
  const float* kk; const float* bk;  // [tokd][A], [A]
  const float* av; const float* ag; const float* ab;  // [A/heads], scalar, [A/heads]
  int ntok, tokd, A, heads;
  float* ref_out;  // [B][128]
  float* style;    // [B][style_w] (writes at style_off)
  int style_w, style_off;
};

__global__ __launch_bounds__(256) void k_ref_gru_gst(RefGstArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int D = a.D;
  float* rh = sm;                 // [D] r * h
  float* h = rh + D;              // [D]
  float* gates = h + D;           // [2D]
  float* ref = gates + 2 * D;     // [128]
  float* q = ref + 128;           // [A]
  float* keys = q + a.A;          // [ntok][A]
  float* vals = keys + a.ntok * a.A;  // [ntok][tokd]
  float* sc = vals + a.ntok * a.tokd; // [heads][ntok]
  for (int i = tid; i < D; i += blockDim.x) h[i] = 0.f;
  __syncthreads();
  // TF GRUCell over every padded frame: [r, u] = σ([x, h]·Wg + bg), c = tanh([x, r⊙h]·Wc + bc),
  // h' = u⊙h + (1-u)⊙c.  The x rows of both kernels (+ biases) were applied to all frames by one
  // GEMM before this kernel; each step only does the D recurrent rows.
  for (int t = 0; t < a.T2; ++t) {
    const float* xg = a.xg + ((long)b * a.T2 + t) * 3 * D;
    for (int j = tid; j < 2 * D; j += blockDim.x) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 4
      for (int k = 0; k < D; k += 4) {
        s0 += h[k] * a.whg[(long)k * 2 * D + j];
        s1 += h[k + 1] * a.whg[(long)(k + 1) * 2 * D + j];
        s2 += h[k + 2] * a.whg[(long)(k + 2) * 2 * D + j];
        s3 += h[k + 3] * a.whg[(long)(k + 3) * 2 * D + j];
      }
      gates[j] = sigm(xg[j] + ((s0 + s1) + (s2 + s3)));
    }
    __syncthreads();
    for (int i = tid; i < D; i += blockDim.x) rh[i] = gates[i] * h[i];
    __syncthreads();
    float hn = 0.f;
    if (tid < D) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 4
      for (int k = 0; k < D; k += 4) {
        s0 += rh[k] * a.whc[(long)k * D + tid];
        s1 += rh[k + 1] * a.whc[(long)(k + 1) * D + tid];
        s2 += rh[k + 2] * a.whc[(long)(k + 2) * D + tid];
        s3 += rh[k + 3] * a.whc[(long)(k + 3) * D + tid];
      }
      const float c = tanhf(xg[2 * D + tid] + ((s0 + s1) + (s2 + s3)));
      const float u = gates[D + tid];
      hn = u * h[tid] + (1.f - u) * c;
    }
    __syncthreads();
    if (tid < D) h[tid] = hn;
    __syncthreads();
  }
  // dense(128, tanh) on the last GRU output
  if (tid < 128) {
    float s = 0.f;
    for (int k = 0; k < D; ++k) s += h[k] * a.kd[k * 128 + tid];
    ref[tid] = tanhf(s + a.bd[tid]);
    a.ref_out[b * 128 + tid] = ref[tid];
  }
  if (!a.tokens) {  // the reference embedding itself: pretrained_emb_disc_all / use_gst=False /
                    // AdaIN (tacotron.py:266-291), or refnet_spk of the emt variant (style null)
    if (a.style && tid < 128) a.style[(long)b * a.style_w + a.style_off + tid] = ref[tid];
    return;
  }
  // GST values = tanh(tokens)
  for (int i = tid; i < a.ntok * a.tokd; i += blockDim.x) vals[i] = tanhf(a.tokens[i]);
  __syncthreads();
  for (int j = tid; j < a.A; j += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < 128; ++k) s += ref[k] * a.kq[k * a.A + j];
    q[j] = s + a.bq[j];
  }
  for (int e = tid; e < a.ntok * a.A; e += blockDim.x) {
    const int tok = e / a.A, j = e % a.A;
    float s = 0.f;
    for (int d = 0; d < a.tokd; ++d) s += vals[tok * a.tokd + d] * a.kk[d * a.A + j];
    keys[e] = s + a.bk[j];
  }
  __syncthreads();
  const int dh = a.A / a.heads;
  // normed_v = g * v * rsqrt(sum(v^2))
  float vn = 0.f;
  for (int d = 0; d < dh; ++d) vn += a.av[d] * a.av[d];
  const float scale = a.ag[0] * (1.0f / sqrtf(vn));
  for (int e = tid; e < a.heads * a.ntok; e += blockDim.x) {
    const int hh = e / a.ntok, tok = e % a.ntok;
    float s = 0.f;
    for (int d = 0; d < dh; ++d)
      s += (scale * a.av[d]) * tanhf(keys[tok * a.A + hh * dh + d] + q[hh * dh + d] + a.ab[d]);
    sc[e] = s;
  }
  __syncthreads();
  if (tid < a.heads) {
    float mx = -INFINITY;
    for (int tok = 0; tok < a.ntok; ++tok) mx = fmaxf(mx, sc[tid * a.ntok + tok]);
    float sum = 0.f;
    for (int tok = 0; tok < a.ntok; ++tok) {
      const float e = expf(sc[tid * a.ntok + tok] - mx);
      sc[tid * a.ntok + tok] = e;
      sum += e;
    }
    for (int tok = 0; tok < a.ntok; ++tok) sc[tid * a.ntok + tok] /= sum;
  }
  __syncthreads();
  for (int e = tid; e < a.heads * a.tokd; e += blockDim.x) {
    const int hh = e / a.tokd, d = e % a.tokd;
    float s = 0.f;
    for (int tok = 0; tok < a.ntok; ++tok) s += sc[hh * a.ntok + tok] * vals[tok * a.tokd + d];
    a.style[(long)b * a.style_w + a.style_off + e] = s;
  }
}

// values = concat(encoder_outputs, tile(style)) · seq_mask (tacotron.py:307-308 + TF
// BahdanauAttention._prepare_memory)
__global__ void k_memory(const float* __restrict__ enc, const float* __restrict__ style,
                         const int* __restrict__ lengths, float* __restrict__ values, int B, int T, int E2,
                         int SW) {
  const int row = blockIdx.x;  // b*T + t
  const int b = row / T, t = row % T;
  const int D = E2 + SW;
  const bool valid = t < lengths[b];
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float v = 0.f;
    if (valid) v = d < E2 ? enc[(long)row * E2 + d] : style[(long)b * SW + d - E2];
    values[(long)row * D + d] = v;
  }
}

// ReferenceEncoderAdaIn (modules.py:89-98): tf.nn.moments(x, axes=[1, 2]) of the NHWC conv output
// x [B][HW][C] per (row, channel), two-pass (mean, then mean squared deviation) -> mv[b][c] = {m, v}
__global__ __launch_bounds__(256) void k_adain_moments(const float* __restrict__ x, int HW, int C,
                                                       float* __restrict__ mv) {
  __shared__ float red[256];
  const int b = blockIdx.x, ch = blockIdx.y, tid = threadIdx.x;
  const float* xb = x + (long)b * HW * C + ch;
  float acc = 0.f;
  for (int i = tid; i < HW; i += 256) acc += xb[(long)i * C];
  red[tid] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const float mean = red[0] / (float)HW;
  __syncthreads();
  acc = 0.f;
  for (int i = tid; i < HW; i += 256) {
    const float d = xb[(long)i * C] - mean;
    acc += d * d;
  }
  red[tid] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) {
    mv[((long)b * C + ch) * 2] = mean;
    mv[((long)b * C + ch) * 2 + 1] = red[0] / (float)HW;
  }
}

// spk = 0.9·spk + 0.1·tf.nn.batch_normalization(spk, mean_spk, var_spk, offset=mean_emt,
// scale=var_emt, 1e-9) (modules.py:94-98): inv = rsqrt(var_s + eps)·var_e, x·inv + (m_e − m_s·inv)
__global__ void k_adain_mix(float* __restrict__ x, long n, int HW, int C, const float* __restrict__ mv_s,
                            const float* __restrict__ mv_e) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int ch = (int)(i % C);
  const long b = i / ((long)HW * C);
  const float* s = mv_s + (b * C + ch) * 2;
  const float* e = mv_e + (b * C + ch) * 2;
  const float inv = (1.0f / sqrtf(s[1] + 1e-9f)) * e[1];
  const float v = x[i];
  x[i] = v * 0.9f + (v * inv + (e[0] - s[0] * inv)) * 0.1f;
}

// ---- decoder -------------------------------------------------------------------------------
//
// One decoder step = 7 dependent launches (captured per 16-step chunk in a hipGraph):
//   k_prenet   finish step t-1 (frame/stop projection reduce, stop rule) + prenet of step t
//   k_lstm     LSTM layer 1 on [prenet | context_enc] (+ precomputed recurrent/style gate terms)
//   k_lstm     LSTM layer 2 on h1_new (+ precomputed recurrent gate term)
//   k_partial  query layer (split-K partials)
//   k_energy   location-sensitive energies          + side job: W_hh2·h2(t)  for step t+1
//   k_softmax  softmax, alignments, context_enc     + side job: W_hh1·h1(t)  for step t+1
//   k_partial  frame/stop projection (split-K partials)
// Two algebraic identities keep bytes off the per-step critical path:
//  * memory = [encoder outputs | tiled style] masked past each row's length (tacotron.py:297-308),
//    so context_style = (Σ_{t<len} align_t)·style: the softmax kernel reads only the encoder half of
//    the values, and the style rows of the LSTM-1 and projection kernels become per-utterance
//    vectors GS = style·W_style scaled by that per-row sum each step;
//  * [x | h]·W = x·W_x + h·W_h: the recurrent halves h(t-1)·W_h do not depend on step t's chain,
//    so they are computed as extra workgroups ("side jobs") of two latency-bound launches of the
//    previous step and added in the LSTM epilogues.

struct DecCtl {
  int done;
  int n_steps;
  int tbase;
  int pad;
};

// A skinny GEMM [32 x K] · [K x 16·ntile] run as extra workgroups of a host launch:
// block j of the job computes 16 columns, output tile-major out[tile][32][16].
struct SideJob {
  const float* X;   // AF [32 x K]
  const float* W;   // WF tiles [ntile][K x 16]
  float* out;       // [ntile][32][16]
  int K, ntile;
  int delay;        // s_sleep(64) repetitions before the side blocks start (~1.7 us each)
};

struct DecArgs {
  DecCtl* ctl;
  int B, T_in, max_iters, T_lim;   // T_lim: GTA target length (0 = free running)
  int nm, P, H, Dm, E2, A, F, KL;  // E2: encoder-output width of the memory (2 x encoder_lstm_units)
  int K1, Kp;                      // LSTM-1 / projection critical input widths
  float zo, one_m_zo;
  int stop_at_any, mask_encoder, cumulative, constraint, monotonic, win;
  int smoothing;  // hp.smoothing: sigmoid normalisation (attention.py:71-80)
  // weights
  const float* pre_b1; const float* pre_w2; const float* pre_b2;
  const float* q_w; const float* loc_cw;  // WF-packed; loc_cw = W_conv·W_loc [KLp taps x A]
  int KLp, Fp;  // location conv taps / filters padded to 16
  const float* va; const float* proj_w; const float* proj_b;
  const float* PS;      // [32][NPF] style·W_proj_style (per utterance), incl. the folded prenet-L1 columns
  const float* TP1;     // [B][T_lim][P] targets·W1 + b1 (GTA) or null
  const float* pre1;    // [32][P] prenet-L1 pre-activations of the last projection (AF-group order)
  // attention memory
  const float* keys;    // [B][T_in][A]
  const float* values;  // [B][T_in][Dm] (only the first E2 channels are read per step)
  const int* lengths;
  // state / activations
  float* X1[2];   // AF [32 x K1] = [prenet | context_enc], by step parity
  float* Xp;      // AF [32 x Kp] = [h2_new | context_enc]
  float* ssum;    // [32] Σ_{t<len} alignments of the last step
  float* Qp;      // [KSQ][32][A]
  float* energy;  // [B][T_in]
  float* cum;     // [B][T_in]
  int* max_att;   // [B]
  float* PP;      // [KSP][32][NPF]: frame/stop columns [0, NPJ), prenet-L1 columns [NPJ, NPJ+P)
  int KSQ, KSP, NPJ, NPF;
  // noise / teacher
  const uint8_t* masks;  // [max_iters][2][B][P] keep bits (injected, or k_gen_masks from the seed)
  uint64_t seed;
  int stamp_step;        // prenet stamps recorded at this decoder step (diagnostic)
  const float* targets;  // [B][T_lim][nm] or null
  long long* stamps;  // diagnostic s_memtime stamps (profiling only; no output depends on them)
  // outputs
  float* frames;  // [B][max_iters * r][nm]
  float* stop;    // [B][max_iters * r]
  float* align;   // [B][T_in][max_iters] or null
};

// Zero-fill of up to ZL_MAX device buffers in ONE launch (decoder / encoder state resets: one
// launch instead of a hipMemsetAsync per buffer, ~5 us each).  Buffers are DevBuf allocations
// (256-byte aligned); 16-byte stores, byte tail by the first threads.
constexpr int ZL_MAX = 24;
struct ZeroList {
  void* p[ZL_MAX];
  unsigned long long n[ZL_MAX];
  int count;
};
__global__ void k_zero_many(ZeroList z) {
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x,
                           stride = (unsigned long long)gridDim.x * blockDim.x;
  for (int i = 0; i < z.count; ++i) {
    uint4* q = reinterpret_cast<uint4*>(z.p[i]);
    const unsigned long long n16 = z.n[i] / 16;
    for (unsigned long long k = t; k < n16; k += stride) q[k] = make_uint4(0u, 0u, 0u, 0u);
    if (t < z.n[i] % 16) reinterpret_cast<unsigned char*>(z.p[i])[n16 * 16 + t] = 0;
  }
}

// Keep bits of the always-on prenet dropout when the caller injects none: counter-based hash of
// (seed, flat index) -> Bernoulli(0.5) (common.h prenet_keep_bit), generated for the whole decode
// in one launch (also the read-back tt2_prenet_keep_bits).
__global__ void k_gen_masks(uint8_t* __restrict__ m, long n, uint64_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    m[i] = prenet_keep_bit(i, seed);
}

constexpr int KSQ_C = 4;  // query split-K
constexpr int KSP_C = 4;  // projection split-K
#define STAMP(i)                                                                         \
  do {                                                                                   \
    if (a.stamps && blockIdx.x == 0 && threadIdx.x == 0)                                 \
      a.stamps[i] = __builtin_amdgcn_s_memtime();                                        \
  } while (0)

// One side-job tile with an NW-wave block: K split over the waves (every weight load in flight
// before the first MFMA when K/(16·NW) k-groups fit the template), LDS reduce (red: NW·512
// floats), tile-major store.
template <int NW, int NPW>
__device__ __forceinline__ void side_tile(const SideJob& j, int tile, float* red, float* G, int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  const int nsg = j.K / 16;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float* Wt = j.W + (long)tile * j.K * 16;
  if constexpr (NPW > 0) skinny_mfma_all<NPW>(j.X, Wt, wave * NPW, acc0, acc1, lane);
  else skinny_mfma(j.X, Wt, wave * nsg / NW, (wave + 1) * nsg / NW, acc0, acc1, lane);
  reduce_waves_32x16<NW>(acc0, acc1, red, G, wave, lane, tid);
  for (int e = tid; e < 512; e += NW * 64) j.out[(long)tile * 512 + e] = G[e];
}
template <int NW = 4>
__device__ __forceinline__ void side_job(const SideJob& j, int blk, float* red, float* G, int tid) {
  // let the host launch's own (latency-critical) loads reach the memory system first
  if (j.delay > 0) for (int i = 0; i < j.delay; ++i) __builtin_amdgcn_s_sleep(64);
  if (j.K == 1024) side_tile<NW, 64 / NW>(j, blk, red, G, tid);
  else side_tile<NW, 0>(j, blk, red, G, tid);
}

// Side job as its own launch (parallel graph branch).
__global__ __launch_bounds__(256) void k_side(const DecCtl* ctl, SideJob sj) {
  __shared__ float red[4 * 512];
  __shared__ float G[512];
  if (ctl->done) return;
  side_job(sj, blockIdx.x, red, G, threadIdx.x);
}

// Prenet (modules.py:346-357) of step t.  Layer 1 is never recomputed here: its pre-activation
// frame_in·W1 + b1 arrives ready — free running, frame·W1 = [h2|ctx]·(W_f·W1) + b_f·W1 was folded
// into the previous step's projection launch, which also reduced it (pre1); with GTA targets it
// was computed for all steps at decode start (TP1); at t = 0 (GO frame) it is b1.  Frames, stop
// tokens and the stop decision of step t-1 were written by that projection launch too.
// Grid: P/16 blocks (layer-2 column tiles) of 16 waves.
constexpr int PRE_T = 1024;
__global__ __launch_bounds__(PRE_T) void k_prenet(DecArgs a, int istep, int t) {
  __shared__ __attribute__((aligned(16))) float h1[32 * 256];   // AF [32][P<=256]
  __shared__ float red[16 * 512];
  __shared__ float G[512];
  __shared__ __attribute__((aligned(16))) uint8_t mk1[32 * 256];
  __shared__ uint8_t mk2[32 * 16];
  // (never assign to a field of `a`: a modified by-value kernel argument is copied to scratch)
  long long* const stp = (a.stamp_step < 0 || t == a.stamp_step) ? a.stamps : nullptr;
#undef STAMP
#define STAMP(i)                                                                         \
  do {                                                                                   \
    if (stp && blockIdx.x == 0 && threadIdx.x == 0) stp[i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  STAMP(0);
  const int done0 = a.ctl->done;
  const int P = a.P, tile = blockIdx.x;
  // ---- issue every load up front (unconditional, clamped indices: a conditional load becomes
  //      a branch that waits for it).  Layer-1 pre-activations come in "AF-group" column order:
  //      position 4g + j holds column 16(g/4) + g%4 + 4j, so one float4 is the AF float4 of
  //      (row m, group g) in h1.  Items (m, g): lanes run over rows (conflict-free AF stores).
  const int G4 = P / 4;
  const int mode1 = t == 0 ? 0 : (a.targets ? 1 : 2);  // GO frame / GTA teacher / folded projection
  const int im = tid & 31;
  f32x4 l1v[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int g = min((tid >> 5) + it * (PRE_T / 32), G4 - 1);
    if (mode1 == 2) {
      l1v[it] = *reinterpret_cast<const f32x4*>(a.pre1 + (long)im * P + 4 * g);
    } else if (mode1 == 1) {
      const int mm = min(im, a.B - 1), tt = min(t - 1, a.T_lim - 1);
      l1v[it] = *reinterpret_cast<const f32x4*>(a.TP1 + ((long)mm * a.T_lim + tt) * P + 4 * g);
    } else {
      l1v[it] = *reinterpret_cast<const f32x4*>(a.pre_b1 + 4 * g);
    }
  }
  const int nsg2 = P / 16;
  const f32x4* W2v = reinterpret_cast<const f32x4*>(a.pre_w2);
  f32x4 w2 = {0.f, 0.f, 0.f, 0.f};
  if (wave < nsg2) w2 = W2v[((long)tile * nsg2 + wave) * 64 + lane];
  const long mrow = (long)t * 2 * a.B * P;
  const bool has_mask = t < a.max_iters;
  const int nch = 32 * P / 16;  // 16-column chunks of layer-1 masks (<= PRE_T)
  uint4 mv = {0u, 0u, 0u, 0u};
  uint8_t m2v = 0;
  if (has_mask && tid < nch) {
    const int m = (tid * 16) / P;
    if (m < a.B) mv = *reinterpret_cast<const uint4*>(a.masks + mrow + (long)tid * 16);
  }
  if (has_mask && tid < 32 * 16) {
    const int m = tid >> 4, j = tid & 15;
    if (m < a.B) m2v = a.masks[mrow + (long)a.B * P + (long)m * P + tile * 16 + j];
  }
  if (done0) return;
  STAMP(1);
  // ---- keep masks -> LDS: layer 1 in AF-group byte order (4x4 byte transpose of each chunk:
  //      byte 4kk + j <- column kk + 4j), layer 2 as loaded ----
  if (tid < nch) {
    const unsigned w[4] = {mv.x, mv.y, mv.z, mv.w};
    unsigned o[4];
    for (int kk = 0; kk < 4; ++kk)
      o[kk] = ((w[0] >> (8 * kk)) & 0xffu) | (((w[1] >> (8 * kk)) & 0xffu) << 8) |
              (((w[2] >> (8 * kk)) & 0xffu) << 16) | (((w[3] >> (8 * kk)) & 0xffu) << 24);
    reinterpret_cast<uint4*>(mk1)[tid] = uint4{o[0], o[1], o[2], o[3]};
  }
  if (tid < 32 * 16) mk2[tid] = m2v;
  __syncthreads();
  STAMP(2);
  // ---- layer 1: relu(pre-activation) * keep / 0.5 ----
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int g = (tid >> 5) + it * (PRE_T / 32);
    if (g >= G4) break;
    const f32x4 x = l1v[it];
    const unsigned mw = reinterpret_cast<const unsigned*>(mk1)[(im * P + 4 * g) >> 2];
    f32x4 hv;
    for (int e = 0; e < 4; ++e) hv[e] = (fmaxf(x[e], 0.f) / 0.5f) * (float)((mw >> (8 * e)) & 0xffu);
    *reinterpret_cast<f32x4*>(h1 + af_idx(im, 16 * (g >> 2) + (g & 3))) = hv;
  }
  __syncthreads();
  STAMP(4);
  // ---- layer 2: this block's 16 columns, one k-group of 16 per wave ----
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (wave < nsg2) skinny_mfma_w<1>(h1 + wave * 2 * 64 * 4, &w2, 1, acc0, acc1, lane);
  reduce_waves_32x16<16>(acc0, acc1, red, G, wave, lane, tid);
  float* X1 = a.X1[istep & 1];
  for (int e = tid; e < 512; e += blockDim.x) {
    const int m = e >> 4, j = e & 15, n = tile * 16 + j;
    const float v = (fmaxf(G[e] + a.pre_b2[n], 0.f) / 0.5f) * (float)mk2[m * 16 + j];
    X1[af_idx(m, n)] = v;
  }
  STAMP(5);
}
#undef STAMP
#define STAMP(i)                                                                         \
  do {                                                                                   \
    if (a.stamps && blockIdx.x == 0 && threadIdx.x == 0)                                 \
      a.stamps[i] = __builtin_amdgcn_s_memtime();                                        \
  } while (0)

// Zoneout-LSTM layer (modules.py:220-248 on TF LSTMCell): block g owns hidden units [4g, 4g+4)
// = 16 gate columns (i,j,f,o × 4).  gates = X·W (K split over 8 waves, all weight loads in flight
// first) + RG (recurrent h(t-1)·W_h, a side job of the previous step) + ssum·GS (style term) + b;
// fused cell/zoneout epilogue.  Writes h_new (the raw LSTM output, the layer's output) into Xo at
// column ho_off and the zoned state into Hz; c in place.
struct LstmArgs {
  long long* stamps = nullptr;
  const DecCtl* ctl;
  const float* X; int K;
  const float* W; const float* b;
  const float* RG;                    // [H/4][32][16] or null
  const float* GS; const float* ssum; // [32][4H] (lstm column order) + [32], or null
  const float* Hprev; float* Hz;      // AF [32 x H] zoned states t-1 / t
  float* c; int H;
  float* Xo; int ho_off;
  float zo, one_m_zo;
};

template <int NPW>
__global__ __launch_bounds__(512) void k_lstm(LstmArgs a) {
  __shared__ float red[8 * 512];
  __shared__ float G[512];
  STAMP(16);
  const int done = a.ctl->done;  // read early, tested once the weight stream is in flight
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nsg = a.K / 16;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float* Wg = a.W + (long)g * a.K * 16;
  if constexpr (NPW > 0) skinny_mfma_all<NPW>(a.X, Wg, wave * NPW, acc0, acc1, lane);
  else skinny_mfma(a.X, Wg, wave * nsg / 8, (wave + 1) * nsg / 8, acc0, acc1, lane);
  // epilogue operands (independent of the GEMM): issue before the reduction
  float rg[4] = {0.f, 0.f, 0.f, 0.f}, gs[4] = {0.f, 0.f, 0.f, 0.f}, cprev = 0.f, hprev = 0.f, sm = 0.f;
  const int m = tid >> 2, uu = tid & 3, u = 4 * g + uu;
  if (tid < 128) {
    if (a.RG)
      for (int q = 0; q < 4; ++q) rg[q] = a.RG[((long)g * 32 + m) * 16 + 4 * q + uu];
    if (a.GS) {
      for (int q = 0; q < 4; ++q) gs[q] = a.GS[(long)m * 4 * a.H + g * 16 + 4 * q + uu];
      sm = a.ssum[m];
    }
    cprev = a.c[(long)m * a.H + u];
    hprev = a.Hprev[af_idx(m, u)];
  }
  STAMP(17);
  if (done) return;
  reduce_waves_32x16<8>(acc0, acc1, red, G, wave, lane, tid);
  STAMP(18);
  if (tid < 128) {
    const float* bb = a.b + g * 16;
    float z[4];
    for (int q = 0; q < 4; ++q) z[q] = ((G[m * 16 + 4 * q + uu] + rg[q]) + sm * gs[q]) + bb[4 * q + uu];
    const float cn = sigm(z[2] + 1.0f) * cprev + sigm(z[0]) * tanhf(z[1]);
    const float hn = sigm(z[3]) * tanhf(cn);
    a.c[(long)m * a.H + u] = a.one_m_zo * cn + a.zo * cprev;
    a.Xo[af_idx(m, a.ho_off + u)] = hn;
    a.Hz[af_idx(m, u)] = a.one_m_zo * hn + a.zo * hprev;
  }
  STAMP(19);
}

static void launch_lstm(const LstmArgs& l, int H, hipStream_t s) {
  const int nsg = l.K / 16;
  const dim3 grid(H / 4), blk(512);
  const int npw = nsg % 8 == 0 ? nsg / 8 : 0;
  if (npw == 18) hipLaunchKernelGGL(k_lstm<18>, grid, blk, 0, s, l);
  else if (npw == 8) hipLaunchKernelGGL(k_lstm<8>, grid, blk, 0, s, l);
  else if (npw == 7) hipLaunchKernelGGL(k_lstm<7>, grid, blk, 0, s, l);  // emt 'multihead': K1 = 896
  else if (npw == 6) hipLaunchKernelGGL(k_lstm<6>, grid, blk, 0, s, l);
  else if (npw == 4) hipLaunchKernelGGL(k_lstm<4>, grid, blk, 0, s, l);
  else if (npw == 2) hipLaunchKernelGGL(k_lstm<2>, grid, blk, 0, s, l);
  else hipLaunchKernelGGL(k_lstm<0>, grid, blk, 0, s, l);
}

// Split-K skinny GEMM writing partial sums: out[ks][m][ldo] (cols tile*16..) for the query layer
// (attention.py:187) and the frame/stop projections (Architecture_wrappers.py:243-247).
struct PartArgs {
  const DecCtl* ctl;
  const float* X; int K;     // AF input
  const float* W;            // [ntile][K x 16 WF]
  float* out; int ldo; int ntile; int KS;
};

template <int NPW>
__global__ __launch_bounds__(256) void k_partial(PartArgs a, SideJob sj) {
  __shared__ float red[4 * 512];
  __shared__ float G[512];
  if ((int)blockIdx.x >= a.ntile * a.KS) {  // extra blocks: side job
    if (a.ctl->done) return;
    side_job(sj, blockIdx.x - a.ntile * a.KS, red, G, threadIdx.x);
    return;
  }
  const int done = a.ctl->done;
  const int tile = blockIdx.x % a.ntile, ks = blockIdx.x / a.ntile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nsg = a.K / 16;
  const int s0 = ks * nsg / a.KS, s1 = (ks + 1) * nsg / a.KS;
  const int n = s1 - s0;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float* Wt = a.W + (long)tile * a.K * 16;
  if constexpr (NPW > 0) skinny_mfma_all<NPW>(a.X, Wt, s0 + wave * NPW, acc0, acc1, lane);
  else skinny_mfma(a.X, Wt, s0 + wave * n / 4, s0 + (wave + 1) * n / 4, acc0, acc1, lane);
  if (done) return;
  reduce_waves_32x16<4>(acc0, acc1, red, G, wave, lane, tid);
  for (int e = tid; e < 512; e += blockDim.x) {
    const int m = e >> 4, c = tile * 16 + (e & 15);
    a.out[((long)ks * 32 + m) * a.ldo + c] = G[e];
  }
}

static void launch_partial(const PartArgs& p, const SideJob& sj, hipStream_t s) {
  const int nsg = p.K / 16;
  const dim3 grid(p.ntile * p.KS + sj.ntile), blk(256);
  const bool even = nsg % (p.KS * 4) == 0;
  const int npw = even ? nsg / (p.KS * 4) : 0;
  if (npw == 4) hipLaunchKernelGGL(k_partial<4>, grid, blk, 0, s, p, sj);
  else if (npw == 6) hipLaunchKernelGGL(k_partial<6>, grid, blk, 0, s, p, sj);
  else if (npw == 2) hipLaunchKernelGGL(k_partial<2>, grid, blk, 0, s, p, sj);
  else if (npw == 8) hipLaunchKernelGGL(k_partial<8>, grid, blk, 0, s, p, sj);
  else hipLaunchKernelGGL(k_partial<0>, grid, blk, 0, s, p, sj);
}

// Frame/stop projection (Architecture_wrappers.py:243-247, modules.py:392-448) with the folded
// prenet layer 1 of the next step, split-K over KS blocks per 16-column tile.  Each block stores
// its partial tile; the last of a tile's KS blocks (arrival ticket, agent-scope release/acquire,
// cdna_hip_programming.md §6 Guideline 16 counter form) reduces the tile, adds the style term
// and bias, and writes frames[t] / stop[t] / pre1; the stop tile's last arriver also applies the
// batch-level stop rule of TacoTestHelper / dynamic_decode (helpers.py:36-59) and sets `done`.
typedef __attribute__((address_space(1))) float gf32;
typedef __attribute__((address_space(1))) unsigned gu32;

struct ProjArgs {
  DecCtl* ctl;
  const float* X; int K;          // AF [32 x Kp] = [h2 | context_enc]
  const float* W;                 // WF tiles [ntile][K x 16]
  float* PP; int ldo; int ntile; int KS;
  unsigned* cnt;                  // [ntile] arrival tickets (zeroed per decode, reset by the last arriver)
  const float* PS; const float* bias; const float* ssum;
  float* pre1;                    // [32][P] prenet-L1 pre-activations (AF-group column order)
  float* frames; float* stop;      // [B][max_iters * r][nm], [B][max_iters * r]
  int B, nm, NPJ, P, max_iters, T_lim, stop_at_any;
  int r, sc;                      // frames per step; first stop column (sc / 16 = the stop tile)
};

template <int NPW>
__global__ __launch_bounds__(256) void k_proj(ProjArgs a, SideJob sj, int t) {
  __shared__ float red[4 * 512];
  __shared__ float G[512];
  __shared__ float stopv[8 * 32];
  __shared__ int s_last;
  if ((int)blockIdx.x >= a.ntile * a.KS) {  // extra blocks: side job
    if (a.ctl->done) return;
    side_job(sj, blockIdx.x - a.ntile * a.KS, red, G, threadIdx.x);
    return;
  }
  const int done = a.ctl->done;
  const int tile = blockIdx.x % a.ntile, ks = blockIdx.x / a.ntile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nsg = a.K / 16;
  const int s0 = ks * nsg / a.KS, s1 = (ks + 1) * nsg / a.KS;
  const int n = s1 - s0;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float* Wt = a.W + (long)tile * a.K * 16;
  if constexpr (NPW > 0) skinny_mfma_all<NPW>(a.X, Wt, s0 + wave * NPW, acc0, acc1, lane);
  else skinny_mfma(a.X, Wt, s0 + wave * n / 4, s0 + (wave + 1) * n / 4, acc0, acc1, lane);
  if (done) return;
  reduce_waves_32x16<4>(acc0, acc1, red, G, wave, lane, tid);
  // ---- arrival ticket (write-through form, Guideline 16 R1): partials stored sc1 and drained,
  //      one ticket add per block, the last arriver reads the partials with sc1 loads ----
  for (int e = tid; e < 512; e += 256) {
    const int m = e >> 4, c = tile * 16 + (e & 15);
    __hip_atomic_store((gf32*)(a.PP + ((long)ks * 32 + m) * a.ldo + c), G[e], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  if (tid == 0) {
    const unsigned tk = __hip_atomic_fetch_add((gu32*)(a.cnt + tile), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == (unsigned)a.KS - 1;
    if (last) __hip_atomic_store((gu32*)(a.cnt + tile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  for (int e = tid; e < 512; e += 256) {
    const int m = e >> 4, c = tile * 16 + (e & 15);
    float v = 0.f;
    for (int k2 = 0; k2 < a.KS; ++k2)
      v += __hip_atomic_load((gf32*)(a.PP + ((long)k2 * 32 + m) * a.ldo + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = (v + a.ssum[m] * a.PS[(long)m * a.ldo + c]) + a.bias[c];
    if (c >= a.NPJ) {
      a.pre1[(long)m * a.P + (c - a.NPJ)] = v;
    } else if (c < a.nm * a.r) {  // frame t·r + c / nm of the step's r (tacotron.py:357 reshape)
      const int f = c / a.nm;
      if (m < a.B) a.frames[((long)m * a.max_iters * a.r + (long)t * a.r + f) * a.nm + (c - f * a.nm)] = v;
    } else if (c >= a.sc && c < a.sc + a.r) {
      stopv[(c - a.sc) * 32 + m] = sigm(v);
    }
  }
  if (a.sc / 16 != tile) return;  // the tile holding the stop columns decides `done`
  __syncthreads();
  if (wave == 0) {
    // TacoTestHelper (helpers.py:40-54): finished = round(stop) [B, r]; reduce_all over the batch
    // axis first, then any (stop_at_any) / all over the step's r frames -- at r = 1 both are "every
    // valid row rounds to 1"
    const bool valid = lane < a.B;
    int any_f = 0, all_f = 1;
    for (int i = 0; i < a.r; ++i) {
      const float sv = valid ? stopv[i * 32 + lane] : 0.f;
      const bool f = valid && rintf(sv) == 1.0f;
      const unsigned long long fb = __ballot(f), vb = __ballot(valid);
      if (valid) a.stop[(long)lane * a.max_iters * a.r + (long)t * a.r + i] = sv;
      any_f |= fb == vb;
      all_f &= fb == vb;
    }
    int dn = a.stop_at_any == 2 ? 0 : (a.stop_at_any ? any_f : all_f);
    if (a.T_lim > 0) dn = t + 1 >= a.T_lim;  // TacoTrainingHelper: time + 1 >= T_targets
    if (t + 1 >= a.max_iters) dn = 1;         // dynamic_decode maximum_iterations
    if (lane == 0 && dn) {
      a.ctl->n_steps = t + 1;
      a.ctl->done = 1;
    }
  }
}

// Location-sensitive energies (attention.py:37-69, 186-215) for 32 encoder steps of one row:
//   q = Σ query partials;  loc = im2col(cum, KL taps)·(W_conv·W_loc) (MFMA, K = taps);
//   e_t = Σ_k v_a[k]·tanh(keys' + q + loc)  (keys' = keys + b_a + b_conv·W_loc, built at encode)
// then the synthesis window constraint and -inf past the row's length (TF _maybe_mask_score).
// 8 waves, one 16-dim attention tile each (A <= 256).  Blocks past B·ceil(T_in/32) run the
// side job.
constexpr int NWE = 8;
__global__ __launch_bounds__(NWE * 64) void k_energy(DecArgs a, SideJob sj) {
  __shared__ __attribute__((aligned(16))) float smE[NWE * 512 + 512];  // A1 | side-job scratch
  __shared__ float q[256];
  __shared__ float win[32 + 64];
  __shared__ float ep[NWE][32];
  float* A1 = smE;  // AF [32 t][KLp taps]
  const int ntt = (a.T_in + 31) / 32, nE = a.B * ntt;
  if ((int)blockIdx.x >= nE) {
    if (a.ctl->done) return;
    side_job<NWE>(sj, blockIdx.x - nE, smE, smE + NWE * 512, threadIdx.x);
    return;
  }
  STAMP(8);
  const int done = a.ctl->done;
  const int b = blockIdx.x / ntt, t0 = (blockIdx.x % ntt) * 32, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int A = a.A, KL = a.KL, KLp = a.KLp, padl = (KL - 1) / 2;
  // prefetch (unconditional, clamped): the keys this lane consumes (<= 2 tiles x 8 rows)
  float kv[2][8];
  const int ntl = A / 16;
  const int tmax = a.T_in - 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tile = min(wave + NWE * i, ntl - 1);
    const int k = tile * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int t = min(t0 + (lane >> 4) * 4 + (r & 3) + (r >> 2) * 16, tmax);
      kv[i][r] = a.keys[((long)b * a.T_in + t) * A + k];
    }
  }
  const f32x4* CWv = reinterpret_cast<const f32x4*>(a.loc_cw);
  const int nkc = KLp / 16;
  f32x4 wcv[2][4];
  float vkv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tile = min(wave + NWE * i, ntl - 1);
    const int k = tile * 16 + (lane & 15);
    vkv[i] = a.va[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) wcv[i][j] = CWv[((long)tile * nkc + min(j, nkc - 1)) * 64 + lane];
  }
  for (int k = tid; k < A; k += blockDim.x) {
    float qp[KSQ_C];
#pragma unroll
    for (int ks = 0; ks < KSQ_C; ++ks) qp[ks] = a.Qp[((long)ks * 32 + b) * A + k];
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < KSQ_C; ++ks) s += qp[ks];
    q[k] = s;
  }
  for (int i = tid; i < 32 + KL - 1; i += blockDim.x) {
    const int t = t0 - padl + i;
    const float v = a.cum[(long)b * a.T_in + min(max(t, 0), tmax)];
    win[i] = (t >= 0 && t < a.T_in) ? v : 0.f;
  }
  if (done) return;
  __syncthreads();
  STAMP(9);
  for (int e = tid; e < 32 * KLp; e += blockDim.x) {
    const int t = e / KLp, tap = e - t * KLp;
    A1[af_idx(t, tap)] = tap < KL ? win[t + tap] : 0.f;
  }
  __syncthreads();
  STAMP(10);
  float e0[4] = {0.f, 0.f, 0.f, 0.f}, e1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tile = wave + NWE * i;
    if (tile >= ntl) break;
    f32x4 l0 = {0.f, 0.f, 0.f, 0.f}, l1 = {0.f, 0.f, 0.f, 0.f};
    skinny_mfma_w<4>(A1, wcv[i], nkc, l0, l1, lane);
    const int k = tile * 16 + (lane & 15);
    const float vk = vkv[i], qk = q[k];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ta = t0 + (lane >> 4) * 4 + r, tb = ta + 16;
      if (ta < a.T_in) e0[r] += vk * tanh_fast(kv[i][r] + qk + l0[r]);
      if (tb < a.T_in) e1[r] += vk * tanh_fast(kv[i][4 + r] + qk + l1[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    e0[r] = sum16(e0[r]);
    e1[r] = sum16(e1[r]);
  }
  STAMP(11);
  if ((lane & 15) == 0)
    for (int r = 0; r < 4; ++r) {
      ep[wave][(lane >> 4) * 4 + r] = e0[r];
      ep[wave][16 + (lane >> 4) * 4 + r] = e1[r];
    }
  __syncthreads();
  if (tid < 32) {
    const int t = t0 + tid;
    if (t < a.T_in) {
      float e = 0.f;
      for (int w = 0; w < NWE; ++w) e += ep[w][tid];
      if (a.constraint) {
        const int pm = a.max_att[b], w = a.win;
        bool masked;
        if (a.monotonic) masked = (t < pm) || (t >= pm + w);
        else masked = (t < pm - (w / 2 + (w % 2 != 0 ? 1 : 0))) || (t >= pm + w / 2);
        if (masked) e = -4294967296.0f;  // -2**32 + 1 in fp32
      }
      if (a.mask_encoder && t >= a.lengths[b]) e = -INFINITY;
      a.energy[(long)b * a.T_in + t] = e;
    }
  }
  STAMP(12);
}


// softmax → alignments, context_enc = alignments · values[:, :, 0:E2] for 64 channels of one row
// (attention.py:10-35, 217-225); the dc==0 block also updates cum/max_att, writes alignments and
// the row's Σ_{t<len} alignments (the scale of the style half of the context).
// Blocks past B·E2/64 run the side job.
__global__ __launch_bounds__(256) void k_softmax_ctx(DecArgs a, int istep, int t_step, SideJob sj) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int ndc = a.E2 / 64, nS = a.B * ndc;
  if ((int)blockIdx.x >= nS) {
    if (a.ctl->done) return;
    side_job(sj, blockIdx.x - nS, sm, sm + 2048, threadIdx.x);
    return;
  }
  const int done = a.ctl->done;
  const int b = blockIdx.x / ndc, dc = blockIdx.x % ndc, tid = threadIdx.x;
  const int T = a.T_in;
  float* al = sm;                      // [T]
  float* red = al + ((T + 3) & ~3);    // [4*16*16]
  __shared__ float s_max, s_sum;
  // values for this block's 64 channels are independent of the softmax: issue them first
  const int tq = tid >> 4, dq = tid & 15;
  const int d = dc * 64 + dq * 4;
  const float* vr = a.values + (long)b * T * a.Dm + d;
  f32x4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int t = tq + 16 * i;
    if (t < T) v[i] = *reinterpret_cast<const f32x4*>(vr + (long)t * a.Dm);
    else v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int i = tid; i < T; i += blockDim.x) al[i] = a.energy[(long)b * T + i];
  if (done) return;
  __syncthreads();
  if (a.smoothing) {  // _smoothing_normalization (attention.py:71-80): sigmoid(e) / sum_j sigmoid(e)
    for (int i = tid; i < T; i += blockDim.x) al[i] = 1.f / (1.f + expf(-al[i]));
    __syncthreads();
    if (tid < 64) {
      float sum = 0.f;
      for (int i = tid; i < T; i += 64) sum += al[i];
      for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
      if (tid == 0) s_sum = sum;
    }
    __syncthreads();
    for (int i = tid; i < T; i += blockDim.x) al[i] = al[i] / s_sum;
  } else {
    if (tid < 64) {
      float mx = -INFINITY;
      for (int i = tid; i < T; i += 64) mx = fmaxf(mx, al[i]);
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      float sum = 0.f;
      for (int i = tid; i < T; i += 64) sum += expf(al[i] - mx);
      for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
      if (tid == 0) { s_max = mx; s_sum = sum; }
    }
    __syncthreads();
    for (int i = tid; i < T; i += blockDim.x) al[i] = expf(al[i] - s_max) / s_sum;
  }
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int t = tq + 16 * i;
    const float w = t < T ? al[t] : 0.f;
    acc[0] += w * v[i][0]; acc[1] += w * v[i][1]; acc[2] += w * v[i][2]; acc[3] += w * v[i][3];
  }
  for (int t = tq + 256; t < T; t += 16) {  // tail for T_in > 256
    const f32x4 x = *reinterpret_cast<const f32x4*>(vr + (long)t * a.Dm);
    const float w = al[t];
    acc[0] += w * x[0]; acc[1] += w * x[1]; acc[2] += w * x[2]; acc[3] += w * x[3];
  }
  for (int j = 0; j < 4; ++j) red[(j * 16 + dq) * 16 + tq] = acc[j];
  __syncthreads();
  if (tid < 64) {
    const int j = tid >> 4, dq2 = tid & 15;
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += red[(j * 16 + dq2) * 16 + i];
    const int dd = dc * 64 + dq2 * 4 + j;
    a.X1[(istep + 1) & 1][af_idx(b, a.P + dd)] = s;
    a.Xp[af_idx(b, a.H + dd)] = s;
  }
  if (dc == 0) {
    const int len = a.lengths[b];
    for (int i = tid; i < T; i += blockDim.x) {
      float* c = a.cum + (long)b * T + i;
      *c = a.cumulative ? al[i] + *c : al[i];
      if (a.align && t_step < a.max_iters) a.align[((long)b * T + i) * a.max_iters + t_step] = al[i];
    }
    if (tid < 64) {
      float best = -INFINITY, ss = 0.f;
      int bi = 0x7fffffff;
      for (int i = tid; i < T; i += 64) {
        if (al[i] > best) { best = al[i]; bi = i; }
        if (i < len) ss += al[i];
      }
      for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
        ss += __shfl_xor(ss, o);
      }
      if (tid == 0) {
        a.max_att[b] = bi;
        a.ssum[b] = ss;
      }
    }
  }
}

// Encoder-step-fastest copies of keys / values for the persistent decoder:
// dst[b][c][t] = src[b][t][c] (t < T, c < C; row stride ld), 0 for T <= t < 256.
// rows [B][C] -> AF [32 x C] (rows >= B untouched): the persistent decoder's step-0 emotion block
__global__ void k_af_rows(const float* __restrict__ src, int C, float* __restrict__ dst) {
  const int b = blockIdx.x;
  for (int n = threadIdx.x; n < C; n += blockDim.x) dst[af_idx(b, n)] = src[(long)b * C + n];
}

__global__ void k_transpose_bt(const float* __restrict__ src, long ld, float* __restrict__ dst, int T, int C, int ldt) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, c0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int t = t0 + r;
    tile[r][tx] = t < T ? src[((long)b * T + t) * ld + c0 + tx] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) dst[((long)b * C + c0 + r) * ldt + t0 + tx] = tile[tx][r];
}

// step-major alignments [B][n][T] -> the reference layout [B][T][ldt] (tower_alignments), columns < n
__global__ void k_align_t(const float* __restrict__ src, int n, int T, long lds, float* __restrict__ dst, long ldt) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, j0 = blockIdx.y * 32, s0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int st = s0 + r, j = j0 + tx;
    tile[r][tx] = (st < n && j < T) ? src[((long)b * lds + st) * T + j] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int j = j0 + r, st = s0 + tx;
    if (j < T && st < n) dst[((long)b * T + j) * ldt + st] = tile[tx][r];
  }
}

// decoder_output clip (tacotron.py:362-363): dst[b][t][n] = clip(src[b][t][n])
// get_output_lengths (tacotron/synthesizer.py:384-387): per row, the first step whose stop
// probability rounds to 1 (np.round = round-half-even = rintf), else n_steps.  One wave per row,
// 64 steps per ballot.
__global__ __launch_bounds__(64) void k_output_lengths(const float* __restrict__ stop, int n_steps, long ld,
                                                       int* __restrict__ lengths) {
  const int b = blockIdx.x, lane = threadIdx.x;
  int found = n_steps;
  for (int t0 = 0; t0 < n_steps; t0 += 64) {
    const int t = t0 + lane;
    const unsigned long long m = __ballot(t < n_steps && rintf(stop[(long)b * ld + t]) == 1.0f);
    if (m) {
      found = t0 + __builtin_ctzll(m);
      break;
    }
  }
  if (lane == 0) lengths[b] = found;
}

__global__ void k_clip_frames(const float* __restrict__ src, long src_bstride, float* __restrict__ dst, int B,
                              int T, int nm, float lo, float hi, int do_clip) {
  const long n = (long)B * T * nm;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = i / ((long)T * nm);
    const long r = i - (long)b * T * nm;
    float v = src[b * src_bstride + r];
    if (do_clip) v = fminf(fmaxf(v, lo), hi);
    dst[i] = v;
  }
}

// ==========================================================================================
// Host side
// ==========================================================================================
static void zero_many(std::initializer_list<std::pair<void*, size_t>> bufs, hipStream_t s) {
  ZeroList z;
  z.count = 0;
  for (const auto& b : bufs) {
    if (!b.first || !b.second) continue;
    TT2_CHECK(z.count < ZL_MAX, TT2_ERR_INVALID_ARG, "zero_many: too many buffers");
    TT2_CHECK((reinterpret_cast<uintptr_t>(b.first) & 15) == 0, TT2_ERR_INVALID_ARG, "zero_many: unaligned buffer");
    z.p[z.count] = b.first;
    z.n[z.count] = b.second;
    ++z.count;
  }
  if (!z.count) return;
  hipLaunchKernelGGL(k_zero_many, dim3(1024), dim3(256), 0, s, z);
  TT2_HIP(hipGetLastError());
}
// ReferenceEncoder strides (2,2) everywhere; ReferenceEncoderAdaIn (2,2),(2,2),(1,1)x4 (tacotron.py:237)
inline int refnet_stride(bool adain, int layer) { return adain && layer >= 2 ? 1 : 2; }

struct RefNetDev {
  DevBuf cw[6], cb[6], bs[6], bh[6];
  DevBuf wx, bx, whg, whc, kd, bd, tok, kq, bq, kk, bk, av, ag, ab;  // wx = [Wg_x | Wc_x], bx = [bg | bc]
  int gin = 0;
};

struct Graph {
  std::vector<hipGraphExec_t> chunks;  // chunk c covers decoder steps [c*S, c*S+S)
  std::tuple<int, int, int, int, const void*, const void*, uint64_t, const void*, const void*, const void*> key;
};

}  // namespace tt2

struct tt2_ctx {
  tt2_config cfg;
  int dev = 0;
  hipStream_t stream = nullptr;
  // the reference encoders run beside the text encoder (independent until k_memory): fork/join
  hipStream_t ref_stream = nullptr;
  hipEvent_t ref_ev[2] = {nullptr, nullptr};
  tt2::WeightMap host;
  bool finalized = false;
  int nm, E, Cenc, U, Dm, E2, A, F, KL, P, H, PC, SW, K1, Kp, NPJ, NPF, KSQ = tt2::KSQ_C, KSP = tt2::KSP_C, KLp, Fp;
  int R = 1;       // outputs_per_step: frames (and stop tokens) per decoder step
  int SC = 0;      // first stop column of the projection (all R stop columns in one 16-column tile)
  int nref;        // reference encoders with their own weights
  int nmel = 0;    // reference mels the encode reads (AdaIN: one encoder, both mels)
  int style_mode = 0;  // 0 GST, 1 reference embeddings, 2 AdaIN (tt2_config.style_mode)
  tt2::DevBuf adain_mv;  // [2][B][C][2] per-channel moments (emt, spk)
  // weights
  tt2::DevBuf emb;
  tt2::DevBuf enc_cw[8], enc_cb[8], enc_bs[8], enc_bh[8];
  tt2::DevBuf enc_wx, enc_bx, enc_wh;
  tt2::RefNetDev ref[2];
  tt2::DevBuf mem_k;
  tt2::DevBuf kpart;  // split-K partials of the small once-per-utterance GEMMs (this ctx's stream)
  // max |w| of the weights the split fp16x3 MFMA kernels keep resident (pre-scaled by KG_SB):
  // the persistent decoder / BiLSTM need < KG_BMAX, larger weights take the fp32-MFMA launch path
  float kg_wmax_dec = 0.f, kg_wmax_enc = 0.f;
  // tt2_decoder_step: row-major copies of the decoder variables (uploaded on first use), scratch
  tt2::DevBuf st_w[16], st_io, st_scratch;
  bool st_ready = false;
  // the persistent decoder's copies of l1_w, l1_wh, l2_w, l2_wh, proj_w, pre-scaled by KG_SB
  tt2::DevBuf pd_l1_w, pd_l1_wh, pd_l2_w, pd_l2_wh, pd_proj_w;
  tt2::DevBuf pd_e_wd;  // emt 'multihead' in the persistent decoder: attn_emt dense as WF tiles (x KG_SB)
  // emt 'simple' in the persistent decoder: the speaker rows of the LSTM-1 kernel ([128][4H], lstm column
  // order) and per utterance refnet_spk·those rows ([32][4H]): the block's constant speaker half as a bias
  tt2::DevBuf l1_wspk, SPK1;
  tt2::DevBuf pre_w1r, pre_b1, pre_w2, pre_b2, q_w;  // pre_w1r: row-major [nm][P] (GTA TP1 GEMM)
  tt2::DevBuf l1_w, l1_wh, l1_ws, l1_b, l2_w, l2_wh, l2_b;  // critical rows / recurrent rows / style rows
  tt2::DevBuf loc_cw, keys_b, va, proj_w, proj_ws, proj_b;
  tt2::DevBuf post_cw[8], post_cb[8], post_bs[8], post_bh[8], post_pw, post_pb;
  // pre-split fp16 planes of the static conv / projection weights (split16 GEMMs, gemm.h SplitB)
  tt2::SplitB enc_cw_s[8], post_cw_s[8], post_pw_s, mem_k_s;
  // Postnet over pre-split padded planes (gemm.h conv_x3): conv 1's weights at Cp = nm rounded to 32,
  // the input planes of conv 1 and two ping-pong plane pairs; post_cx = 0 runs the im2col GEMMs
  tt2::SplitB post_cx0_s;
  tt2::DevBuf px_in_h, px_in_l, px_h[2], px_l[2];
  bool post_cx = false;
  // text encoder over the same planes (conv_x3 with split K), BiLSTM input projection as a width-1
  // conv; enc_cx = 0 runs the im2col GEMMs
  tt2::SplitB enc_wx_s;
  tt2::DevBuf ex_h[2], ex_l[2], ex_part;
  bool enc_cx = false;
  // activations
  tt2::DevBuf refxg;  // reference-encoder GRU input projections [B][T2][3D]
  tt2::DevBuf enc_hg;  // persistent BiLSTM h granules [2][2][32 x U] + timeout word
  bool enc_err_check = false;
  tt2::DevBuf ids, lens, refm[2], x_a, x_b, xproj, enc_out, enc_h, enc_c, conv_a, conv_b, ref_out, style,
      values, keys;
  tt2::DevBuf X1[2], X2, Xp, H0s[2], H1s[2], RG0, RG1, GS0, PS, ssum, TP1, pre1, pcnt, c1, c2, Qp, energy, cum, max_att, PP, ctl,
      masks, gmasks, targets;
  tt2::DevBuf frames, stop, align, dec, post_a, post_b, mel;
  int* ctl_host = nullptr;  // pinned [2 slots]
  int B = 0, T_in = 0, n_steps = 0, last_max_iters = 0;
  bool encoded = false, decoded = false;
  tt2::Graph graph;
  static constexpr int S = 16;  // decoder steps per captured graph chunk
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // synthesize phase timing
  bool timed = false;
  tt2::DecArgs last_args;
  long long stamps_host[64] = {0};
  int side_mode = 0;                 // TT2_SIDE_MODE env: 0 hosted side jobs, 1 parallel branch
  int side_delay = 1, side_delay2 = 0;  // TT2_SIDE_DELAY / TT2_SIDE_DELAY2 env (energy / softmax host)
  hipEvent_t sev[8] = {nullptr};     // capture-time fork/join events
  bool have_args = false;
  // persistent decoder (decode_persist.hip)
  int pd_mode = 1;        // TT2_DECODER env: 1 persistent when the shapes fit, 0 launch path only
  bool pd_dev_ok = false; // all PD_NB work-groups can be resident on this device
  bool last_pd = false;   // the last decode ran the persistent kernel
  tt2::DevBuf q_wt, pre_w2t, keysT, valuesT, pd_ctl, H1x, H2x, Ex, CTXx, SSx, PPx, PREx, QEx, CMBx, EOx, EMTx;
  tt2::DevBuf pd_alnT;  // [B][max_iters][T_in] step-major alignments of the persistent decoder
  // Tacotron_emt_attn variant (emt.h): off for the Tacotron model
  tt2::EmtModel emt;
  tt2::CbhgModel cbhg;  // predict_linear post-processing net (cbhg.h)
  std::vector<int> emt_labels;  // tt2_set_emt_labels (style_tokens)
  hipEvent_t pd_ev[2] = {nullptr, nullptr};
  float pd_kernel_ms = 0.f;
};

namespace tt2 {

static void upload(DevBuf& d, const std::vector<float>& h) {
  d.alloc(h.size() * sizeof(float));
  TT2_HIP(hipMemcpy(d.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
}
static void upload(DevBuf& d, const HostTensor& t) { upload(d, t.data); }
static void upload_scaled(DevBuf& d, std::vector<float> h, float scale) {
  for (float& x : h) x *= scale;  // exact: power of two
  upload(d, h);
}
static float absmax(const std::vector<float>& v) {
  float m = 0.f;
  for (float x : v) m = std::max(m, std::fabs(x));
  return m;
}

// BN inference constants: y*scale + shift with scale = gamma·rsqrt(var+eps), shift = beta − mean·scale
static void bn_consts(const WeightMap& wm, const std::string& scope, int c, DevBuf& sc, DevBuf& sh) {
  const auto& g = need(wm, scope + "batch_normalization/gamma", {c});
  const auto& be = need(wm, scope + "batch_normalization/beta", {c});
  const auto& m = need(wm, scope + "batch_normalization/moving_mean", {c});
  const auto& v = need(wm, scope + "batch_normalization/moving_variance", {c});
  std::vector<float> s(c), h(c);
  for (int i = 0; i < c; ++i) {
    s[i] = g.data[i] / sqrtf(v.data[i] + 1e-3f);
    h[i] = be.data[i] - m.data[i] * s[i];
  }
  upload(sc, s);
  upload(sh, h);
}

// Repack W[K][N] columns `cols` (16 per tile) into WF tiles, K padded to Kp (zeros)
static std::vector<float> pack_wf(const float* W, int K, int N, const std::vector<int>& cols, int Kp) {
  const int nt = (int)cols.size() / 16;
  std::vector<float> out((size_t)nt * Kp * 16, 0.f);
  for (int tile = 0; tile < nt; ++tile)
    for (int j = 0; j < 16; ++j) {
      const int c = cols[tile * 16 + j];
      if (c < 0) continue;
      for (int k = 0; k < K; ++k) out[(size_t)tile * Kp * 16 + wf_idx(k, j)] = W[(size_t)k * N + c];
    }
  return out;
}

// AF-group column order of the prenet layer-1 pre-activations: position p = 4g + j holds column
// 16(g/4) + g%4 + 4j, so a float4 at 4g is the AF float4 of group g (k_prenet)
static int af_group_col(int p) {
  const int g = p >> 2, j = p & 3;
  return 16 * (g >> 2) + (g & 3) + 4 * j;
}

// LSTM gate column order per block g: [i u0..u3, j u0..u3, f u0..u3, o u0..u3]
static std::vector<int> lstm_cols(int H) {
  std::vector<int> cols;
  for (int g = 0; g < H / 4; ++g)
    for (int gate = 0; gate < 4; ++gate)
      for (int uu = 0; uu < 4; ++uu) cols.push_back(gate * H + 4 * g + uu);
  return cols;
}

// the persistent decoder's tile order: tile g owns units pd_unit(g, 0..3) (decode_persist.h)
static std::vector<int> pd_lstm_cols(int H) {
  std::vector<int> cols;
  for (int g = 0; g < H / 4; ++g)
    for (int gate = 0; gate < 4; ++gate)
      for (int uu = 0; uu < 4; ++uu) cols.push_back(gate * H + pd_unit(g, uu));
  return cols;
}

static void finalize(tt2_ctx* c) {
  const auto& cfg = c->cfg;
  const WeightMap& wm = c->host;
  const std::string P(TP);
  TT2_HIP(hipSetDevice(c->dev));
  upload(c->emb, need(wm, P + "inputs_embedding", {cfg.n_symbols, c->E}));
  int cin = c->E;
  for (int i = 1; i <= cfg.enc_conv_num_layers; ++i) {
    const std::string s = P + "encoder_convolutions/conv_layer_" + std::to_string(i) + "_encoder_convolutions/";
    upload(c->enc_cw[i - 1], need(wm, s + "conv1d/kernel", {cfg.enc_conv_kernel_size, cin, c->Cenc}));
    split_weights(c->enc_cw[i - 1].as<float>(), cfg.enc_conv_kernel_size * cin, c->Cenc, c->Cenc, c->enc_cw_s[i - 1],
                  nullptr);
    upload(c->enc_cb[i - 1], need(wm, s + "conv1d/bias", {c->Cenc}));
    bn_consts(wm, s, c->Cenc, c->enc_bs[i - 1], c->enc_bh[i - 1]);
    cin = c->Cenc;
  }
  {
    const int U = c->U;
    std::vector<float> wx((size_t)cin * 8 * U), bx(8 * U);
    std::vector<float> wh;
    for (int d = 0; d < 2; ++d) {
      const std::string s = P + "encoder_LSTM/bidirectional_rnn/" + (d ? "bw" : "fw") + "/lstm_cell/";
      const auto& k = need(wm, s + "kernel", {cin + U, 4 * U});
      const auto& b = need(wm, s + "bias", {4 * U});
      for (int r = 0; r < cin; ++r)
        for (int col = 0; col < 4 * U; ++col) wx[(size_t)r * 8 * U + d * 4 * U + col] = k.data[(size_t)r * 4 * U + col];
      for (int col = 0; col < 4 * U; ++col) bx[d * 4 * U + col] = b.data[col];
      auto p = pack_wf(k.data.data() + (size_t)cin * 4 * U, U, 4 * U, lstm_cols(U), U);
      wh.insert(wh.end(), p.begin(), p.end());
    }
    upload(c->enc_wx, wx);
    upload(c->enc_bx, bx);
    if (c->enc_cx) split_weights(c->enc_wx.as<float>(), cin, 8 * U, 8 * U, c->enc_wx_s, nullptr);
    upload(c->enc_wh, wh);
    c->kg_wmax_enc = absmax(wh);
  }
  // reference encoders + GST (emt variant: convolutions of refnet_emt, whose outputs emt.hip
  // consumes, and refnet_spk's GRU + dense; no style tokens)
  const char* tags[2] = {"emt", "spk"};
  const bool emt_model = c->emt.on();
  const bool adain = c->style_mode == 2;  // one 'refnet' without batch norm (modules.py:66-107)
  for (int r = 0; r < c->nref; ++r) {
    auto& R = c->ref[r];
    const std::string s = P + (adain ? std::string("refnet") : std::string("refnet_") + tags[r]) + "/";
    int ci = 1, F = cfg.num_mels;
    for (int i = 0; i < 6; ++i) {
      const std::string s2 = s + "conv2d_" + std::to_string(i) + "/";
      const int f = cfg.reference_filters[i];
      upload(R.cw[i], need(wm, s2 + "conv2d/kernel", {3, 3, ci, f}));
      upload(R.cb[i], need(wm, s2 + "conv2d/bias", {f}));
      if (!adain) bn_consts(wm, s2, f, R.bs[i], R.bh[i]);
      ci = f;
      if (refnet_stride(adain, i) == 2) F = (F + 1) / 2;
    }
    const int gin = F * ci, D = cfg.reference_depth;
    R.gin = gin;
    if (adain) {  // the emotion stack's own convs: conv2d_i/conv2d_1/* (tf.layers default-name
                  // uniquification in the re-entered scope, modules.py:84-87) -> ref[1]
      int ce = 1;
      for (int i = 0; i < 6; ++i) {
        const std::string s2 = s + "conv2d_" + std::to_string(i) + "/";
        const int f = cfg.reference_filters[i];
        upload(c->ref[1].cw[i], need(wm, s2 + "conv2d_1/kernel", {3, 3, ce, f}));
        upload(c->ref[1].cb[i], need(wm, s2 + "conv2d_1/bias", {f}));
        ce = f;
      }
    }
    if (emt_model && r == 0) continue;
    {
      const auto& kg = need(wm, s + "rnn/gru_cell/gates/kernel", {gin + D, 2 * D});
      const auto& bg = need(wm, s + "rnn/gru_cell/gates/bias", {2 * D});
      const auto& kc = need(wm, s + "rnn/gru_cell/candidate/kernel", {gin + D, D});
      const auto& bc = need(wm, s + "rnn/gru_cell/candidate/bias", {D});
      std::vector<float> wx((size_t)gin * 3 * D), bx(3 * D);
      for (int k = 0; k < gin; ++k) {
        for (int j = 0; j < 2 * D; ++j) wx[(size_t)k * 3 * D + j] = kg.data[(size_t)k * 2 * D + j];
        for (int j = 0; j < D; ++j) wx[(size_t)k * 3 * D + 2 * D + j] = kc.data[(size_t)k * D + j];
      }
      for (int j = 0; j < 2 * D; ++j) bx[j] = bg.data[j];
      for (int j = 0; j < D; ++j) bx[2 * D + j] = bc.data[j];
      upload(R.wx, wx);
      upload(R.bx, bx);
      upload(R.whg, std::vector<float>(kg.data.begin() + (size_t)gin * 2 * D, kg.data.end()));
      upload(R.whc, std::vector<float>(kc.data.begin() + (size_t)gin * D, kc.data.end()));
      R.gin = gin;
    }
    upload(R.kd, need(wm, s + "dense/kernel", {D, 128}));
    upload(R.bd, need(wm, s + "dense/bias", {128}));
    if (emt_model || c->style_mode != 0) continue;
    const int tokd = cfg.style_embed_depth / cfg.num_heads, Aa = cfg.style_att_dim;
    upload(R.tok, need(wm, P + "style_tokens_" + tags[r], {cfg.num_gst, tokd}));
    const std::string mh = P + "Multihead-attention-" + tags[r] + "/";
    upload(R.kq, need(wm, mh + "conv1d/kernel", {1, 128, Aa}));
    upload(R.bq, need(wm, mh + "conv1d/bias", {Aa}));
    upload(R.kk, need(wm, mh + "conv1d_1/kernel", {1, tokd, Aa}));
    upload(R.bk, need(wm, mh + "conv1d_1/bias", {Aa}));
    upload(R.av, need(wm, mh + "attention_v", {Aa / cfg.num_heads}));
    upload(R.ag, need(wm, mh + "attention_g", {}));
    upload(R.ab, need(wm, mh + "attention_b", {Aa / cfg.num_heads}));
  }
  emt_load(c->emt, wm, P);
  if (cfg.predict_linear) {
    cbhg_load(c->cbhg, wm, P, c->nm, cfg.cbhg_kernels, cfg.cbhg_conv_channels, cfg.cbhg_pool_size, cfg.cbhg_projection,
              cfg.cbhg_projection_kernel_size, cfg.cbhg_highwaynet_layers, cfg.cbhg_highway_units, cfg.cbhg_rnn_units,
              cfg.num_freq);
    c->cbhg.clip = cfg.clip_outputs;
    c->cbhg.clip_lo = cfg.symmetric_mels ? -cfg.max_abs_value - cfg.lower_bound_decay : -cfg.lower_bound_decay;
    c->cbhg.clip_hi = cfg.max_abs_value;
  }
  upload(c->mem_k, need(wm, P + "memory_layer/kernel", {c->Dm, c->A}));
  split_weights(c->mem_k.as<float>(), c->Dm, c->A, c->A, c->mem_k_s, nullptr);
  c->kpart.alloc(sizeof(float) * (8u << 20));
  // decoder
  {
    std::vector<int> cols;
    for (int j = 0; j < c->P; ++j) cols.push_back(j);
    // layer 1 in AF-group column order (see k_prenet): used for the GTA TP1 GEMM and the GO frame
    const auto& w1 = need(wm, P + "decoder/decoder_prenet/dense_1/kernel", {c->nm, c->P});
    const auto& b1 = need(wm, P + "decoder/decoder_prenet/dense_1/bias", {c->P});
    std::vector<float> w1p((size_t)c->nm * c->P), b1p(c->P);
    for (int p = 0; p < c->P; ++p) {
      const int j = af_group_col(p);
      b1p[p] = b1.data[j];
      for (int n = 0; n < c->nm; ++n) w1p[(size_t)n * c->P + p] = w1.data[(size_t)n * c->P + j];
    }
    upload(c->pre_w1r, w1p);
    upload(c->pre_b1, b1p);
    const auto& w2 = need(wm, P + "decoder/decoder_prenet/dense_2/kernel", {c->P, c->P});
    upload(c->pre_w2, pack_wf(w2.data.data(), c->P, c->P, cols, c->P));
    upload(c->pre_b2, need(wm, P + "decoder/decoder_prenet/dense_2/bias", {c->P}));
    std::vector<float> w2t((size_t)c->P * c->P);  // [out][in] for the persistent decoder
    for (int k = 0; k < c->P; ++k)
      for (int n = 0; n < c->P; ++n) w2t[(size_t)n * c->P + k] = w2.data[(size_t)k * c->P + n];
    upload(c->pre_w2t, w2t);
  }
  for (int l = 0; l < 2; ++l) {
    // layer 1 rows: [prenet P | context_enc E2 | context_style SW | h H]; layer 2 rows: [h1_new H | h H]
    const std::string s = P + "decoder/decoder_LSTM/multi_rnn_cell/cell_" + std::to_string(l) + "/lstm_cell/";
    const int H = c->H, N = 4 * H;
    // layer-1 rows: [prenet | context (enc, style) | emotion block (emt variant) | h]
    const int Kfull = l == 0 ? c->P + c->Dm + c->emt.XW + H : 2 * H;
    const int Kc = l == 0 ? c->K1 : H;   // critical rows
    const int Kh0 = l == 0 ? c->K1 + c->SW : H;  // first recurrent row
    const auto& k = need(wm, s + "kernel", {Kfull, N});
    const auto& b = need(wm, s + "bias", {N});
    auto cols = lstm_cols(H);
    std::vector<float> bt(cols.size());
    for (size_t i = 0; i < cols.size(); ++i) bt[i] = b.data[cols[i]];
    {
      const auto wc = pack_wf(k.data.data(), Kc, N, cols, Kc);
      const auto wr = pack_wf(k.data.data() + (size_t)Kh0 * N, H, N, cols, H);
      if (l == 0) c->kg_wmax_dec = 0.f;
      c->kg_wmax_dec = std::max(c->kg_wmax_dec, std::max(absmax(wc), absmax(wr)));
      upload(l == 0 ? c->l1_w : c->l2_w, wc);
      upload(l == 0 ? c->l1_wh : c->l2_wh, wr);
      if (H % 16 == 0) {  // persistent decoder tiles (pd_fits also requires H == PD_H)
        const auto pc = pd_lstm_cols(H);
        upload_scaled(l == 0 ? c->pd_l1_w : c->pd_l2_w, pack_wf(k.data.data(), Kc, N, pc, Kc), KG_SB);
        upload_scaled(l == 0 ? c->pd_l1_wh : c->pd_l2_wh, pack_wf(k.data.data() + (size_t)Kh0 * N, H, N, pc, H), KG_SB);
      }
    }
    upload(l == 0 ? c->l1_b : c->l2_b, bt);
    if (l == 0 && c->emt.attn == EMT_SIMPLE && c->emt.spk) {  // 'simple': [ctx_emt | spk] block, speaker rows
      std::vector<float> wsp((size_t)EMT_OUT * N);
      for (int r = 0; r < EMT_OUT; ++r)
        for (int i = 0; i < N; ++i) wsp[(size_t)r * N + i] = k.data[(size_t)(c->P + c->E2 + c->emt.Aq + r) * N + cols[i]];
      upload(c->l1_wspk, wsp);
    }
    if (l == 0 && c->SW) {  // style rows, lstm column order, row-major [SW][4H] (B operand of the GS GEMM)
      std::vector<float> ws((size_t)c->SW * N);
      for (int r = 0; r < c->SW; ++r)
        for (int i = 0; i < N; ++i) ws[(size_t)r * N + i] = k.data[(size_t)(c->P + c->E2 + r) * N + cols[i]];
      upload(c->l1_ws, ws);
    }
  }
  {
    std::vector<int> cols;
    for (int j = 0; j < c->A; ++j) cols.push_back(j);
    const auto& q = need(wm, P + "decoder/query_layer/kernel", {c->H, c->A});
    upload(c->q_w, pack_wf(q.data.data(), c->H, c->A, cols, c->H));
    std::vector<float> qt((size_t)c->A * c->H);  // [A][H]: the persistent decoder's per-row query slices
    for (int k = 0; k < c->H; ++k)
      for (int n = 0; n < c->A; ++n) qt[(size_t)n * c->H + k] = q.data[(size_t)k * c->A + n];
    upload(c->q_wt, qt);
  }
  const std::string la = P + "decoder/Location_Sensitive_Attention/";
  {
    // location features (attention.py:37-69): conv [KL][1][F] then dense [F][A], both linear, are
    // folded into one [KL x A] filter (A/16 WF tiles over K = KLp taps); the conv bias·W_loc and
    // the attention bias b_a join the keys (memory_layer output) as one per-dim bias
    const auto& cw = need(wm, la + "location_features_convolution/kernel", {c->KL, 1, c->F});
    const auto& cb = need(wm, la + "location_features_convolution/bias", {c->F});
    const auto& lw = need(wm, la + "location_features_layer/kernel", {c->F, c->A});
    const auto& ba = need(wm, la + "attention_bias", {c->A});
    std::vector<float> wc((size_t)c->KL * c->A), kb(c->A);
    for (int k = 0; k < c->A; ++k) {
      for (int tap = 0; tap < c->KL; ++tap) {
        double acc = 0.0;
        for (int f = 0; f < c->F; ++f) acc += (double)cw.data[(size_t)tap * c->F + f] * lw.data[(size_t)f * c->A + k];
        wc[(size_t)tap * c->A + k] = (float)acc;
      }
      double bacc = 0.0;
      for (int f = 0; f < c->F; ++f) bacc += (double)cb.data[f] * lw.data[(size_t)f * c->A + k];
      kb[k] = (float)(bacc + ba.data[k]);
    }
    std::vector<int> acols;
    for (int j = 0; j < c->A; ++j) acols.push_back(j);
    upload(c->loc_cw, pack_wf(wc.data(), c->KL, c->A, acols, c->KLp));
    upload(c->keys_b, kb);
  }
  upload(c->va, need(wm, la + "attention_variable_projection", {c->A}));
  {
    const std::string fp = P + "decoder/linear_transform_projection/projection_linear_transform_projection/";
    const std::string sp = P + "decoder/stop_token_projection/projection_stop_token_projection/";
    // FrameProjection(num_mels * r) / StopProjection(shape=r) (tacotron.py:322-324)
    const int r = c->R, NF = c->nm * r;
    const auto& fk = need(wm, fp + "kernel", {c->H + c->Dm, NF});
    const auto& fb = need(wm, fp + "bias", {NF});
    const auto& sk = need(wm, sp + "kernel", {c->H + c->Dm, r});
    const auto& sb = need(wm, sp + "bias", {r});
    // columns [0, NPJ): frames (nm·r) | 0-pad | stop (r, from SC) | 0-pad; [NPJ, NPF): prenet layer 1
    // folded through the LAST frame's projection columns, W_f[:, (r-1)·nm:]·W1 (free-running decoding
    // feeds the step's last frame back: helpers.py:57)
    const int N = NF + r, Kfull = c->H + c->Dm, NPF = c->NPF, Pn = c->P, l0 = (r - 1) * c->nm;
    const auto& w1 = need(wm, P + "decoder/decoder_prenet/dense_1/kernel", {c->nm, Pn});
    const auto& b1 = need(wm, P + "decoder/decoder_prenet/dense_1/bias", {Pn});
    std::vector<float> W((size_t)Kfull * NPF, 0.f);
    for (int k = 0; k < Kfull; ++k) {
      for (int n = 0; n < NF; ++n) W[(size_t)k * NPF + n] = fk.data[(size_t)k * NF + n];
      for (int i = 0; i < r; ++i) W[(size_t)k * NPF + c->SC + i] = sk.data[(size_t)k * r + i];
      for (int p = 0; p < Pn; ++p) {
        const int j = af_group_col(p);
        double acc = 0.0;
        for (int n = 0; n < c->nm; ++n) acc += (double)fk.data[(size_t)k * NF + l0 + n] * w1.data[(size_t)n * Pn + j];
        W[(size_t)k * NPF + c->NPJ + p] = (float)acc;
      }
    }
    std::vector<int> cols;
    for (int j = 0; j < NPF; ++j) cols.push_back(j);
    {
      const auto pw = pack_wf(W.data(), c->Kp, NPF, cols, c->Kp);  // rows [h2 | context_enc]
      c->kg_wmax_dec = std::max(c->kg_wmax_dec, absmax(pw));
      upload(c->proj_w, pw);
      const bool emt_mh = c->emt.on();
      if (emt_mh && c->emt.Aq == PD_EQ) {
        // persistent decoder: 8 more tiles = the emotion query h2·W_q (multihead conv1d, first H rows --
        // 'style_tokens' appends the one-hot label rows, folded into the per-row query bias; zero context
        // rows), Architecture_wrappers.py:228-232 / multihead_attention.py:71
        const int qin = c->H + (c->emt.attn == EMT_STYLE_TOKENS ? c->emt.n_emt : 0);
        // 'simple': the query is W2(h2) (attention.py:241-250)
        const auto& kq = c->emt.attn == EMT_SIMPLE ? need(wm, P + "decoder/W2/kernel", {c->H, PD_EQ})
                                                    : need(wm, P + "decoder/Multihead-attention-attn_emt/conv1d/kernel", {1, qin, PD_EQ});
        const int NX = NPF + PD_EQ;
        std::vector<float> Wx((size_t)c->Kp * NX, 0.f);
        std::vector<int> colx;
        for (int j = 0; j < NX; ++j) colx.push_back(j);
        for (int k = 0; k < c->Kp; ++k) {
          for (int n = 0; n < NPF; ++n) Wx[(size_t)k * NX + n] = W[(size_t)k * NPF + n];
          if (k < c->H)
            for (int n = 0; n < PD_EQ; ++n) Wx[(size_t)k * NX + NPF + n] = kq.data[(size_t)k * PD_EQ + n];
        }
        const auto pwx = pack_wf(Wx.data(), c->Kp, NX, colx, c->Kp);
        c->kg_wmax_dec = std::max(c->kg_wmax_dec, absmax(pwx));
        upload_scaled(c->pd_proj_w, pwx, KG_SB);
        if (c->emt.attn == EMT_MULTIHEAD) {  // the attn_emt dense as WF tiles ('style_tokens' has none)
          const int KC = c->emt.heads * c->emt.Dv;
          const auto& kd = need(wm, P + "decoder/attn_emt/dense/kernel", {KC, EMT_OUT});
          std::vector<int> ocols;
          for (int j = 0; j < EMT_OUT; ++j) ocols.push_back(j);
          const auto pwd = pack_wf(kd.data.data(), KC, EMT_OUT, ocols, KC);
          c->kg_wmax_dec = std::max(c->kg_wmax_dec, absmax(pwd));
          upload_scaled(c->pd_e_wd, pwd, KG_SB);
        }
      } else {
        upload_scaled(c->pd_proj_w, pw, KG_SB);
      }
    }
    std::vector<float> ws((size_t)c->SW * NPF, 0.f);                // context_style rows
    for (int r = 0; r < c->SW; ++r)
      for (int n = 0; n < NPF; ++n) ws[(size_t)r * NPF + n] = W[(size_t)(c->Kp + r) * NPF + n];
    if (c->SW) upload(c->proj_ws, ws);
    std::vector<float> pb(NPF, 0.f);
    for (int n = 0; n < NF; ++n) pb[n] = fb.data[n];
    for (int i = 0; i < r; ++i) pb[c->SC + i] = sb.data[i];
    for (int p = 0; p < Pn; ++p) {  // b_f[(r-1)·nm:]·W1 + b1
      const int j = af_group_col(p);
      double acc = 0.0;
      for (int n = 0; n < c->nm; ++n) acc += (double)fb.data[l0 + n] * w1.data[(size_t)n * Pn + j];
      pb[c->NPJ + p] = (float)(acc + b1.data[j]);
    }
    upload(c->proj_b, pb);
    (void)N;
  }
  cin = c->nm;
  for (int i = 1; i <= cfg.postnet_num_layers; ++i) {
    const std::string s = P + "postnet_convolutions/conv_layer_" + std::to_string(i) + "_postnet_convolutions/";
    upload(c->post_cw[i - 1], need(wm, s + "conv1d/kernel", {cfg.postnet_kernel_size, cin, c->PC}));
    split_weights(c->post_cw[i - 1].as<float>(), cfg.postnet_kernel_size * cin, c->PC, c->PC, c->post_cw_s[i - 1],
                  nullptr);
    upload(c->post_cb[i - 1], need(wm, s + "conv1d/bias", {c->PC}));
    bn_consts(wm, s, c->PC, c->post_bs[i - 1], c->post_bh[i - 1]);
    cin = c->PC;
  }
  upload(c->post_pw, need(wm, P + "postnet_projection/projection_postnet_projection/kernel", {c->PC, c->nm}));
  split_weights(c->post_pw.as<float>(), c->PC, c->nm, c->nm, c->post_pw_s, nullptr);
  if (c->post_cx)
    split_conv_weights(c->post_cw[0].as<float>(), cfg.postnet_kernel_size, c->nm, (c->nm + 31) / 32 * 32, c->PC,
                       c->post_cx0_s, nullptr);
  TT2_HIP(hipDeviceSynchronize());
  upload(c->post_pb, need(wm, P + "postnet_projection/projection_postnet_projection/bias", {c->nm}));
  c->finalized = true;
  c->st_ready = false;
}

// K split of the text-encoder convolutions on the planes path (TT2_ENC_SPLITK, 1..8; default 4)
constexpr int kEncSplitK = 8;
static int enc_split_k() {
  const char* e = std::getenv("TT2_ENC_SPLITK");
  return e ? std::max(1, std::min(kEncSplitK, std::atoi(e))) : 4;
}

static void alloc_acts(tt2_ctx* c) {
  const auto& cfg = c->cfg;
  const long B = cfg.max_batch, T = cfg.max_T_in, TR = std::max(cfg.max_T_ref, 1), MI = cfg.max_iters;
  const long W = std::max<long>({(long)c->E, (long)c->Cenc});
  c->ids.alloc(B * T * 4);
  c->lens.alloc(64 * 4);
  for (int r = 0; r < 2; ++r) c->refm[r].alloc(B * TR * c->nm * 4);
  c->x_a.alloc(B * T * W * 4);
  c->x_b.alloc(B * T * W * 4);
  c->xproj.alloc(B * T * 8 * c->U * 4);
  c->enc_out.alloc(B * T * 2 * c->U * 4);
  c->enc_h.alloc(4L * 32 * c->U * 4);
  c->enc_c.alloc(2L * 32 * c->U * 4);
  // refnet conv scratch: largest layer output = B * ceil(T/2) * ceil(80/2) * filters[0..1]
  long mx = 0;
  {
    long t = TR, f = c->nm;
    for (int i = 0; i < 6; ++i) {
      if (refnet_stride(c->style_mode == 2, i) == 2) {
        t = (t + 1) / 2;
        f = (f + 1) / 2;
      }
      mx = std::max(mx, B * t * f * cfg.reference_filters[i]);
    }
  }
  if (c->style_mode == 2) c->adain_mv.alloc(sizeof(float) * 2 * B * cfg.reference_filters[5] * 2);
  c->conv_a.alloc(std::max(mx, 16L) * 4);
  c->conv_b.alloc(std::max(mx, 16L) * 4);
  c->ref_out.alloc(2 * B * 128 * 4);
  c->style.alloc(B * std::max(c->SW, 1) * 4);
  c->values.alloc(B * T * c->Dm * 4);
  c->keys.alloc(B * T * c->A * 4);
  for (int p = 0; p < 2; ++p) {
    c->X1[p].alloc(32L * c->K1 * 4);
    c->H0s[p].alloc(32L * c->H * 4);
    c->H1s[p].alloc(32L * c->H * 4);
  }
  c->X2.alloc(32L * c->H * 4);
  c->Xp.alloc(32L * c->Kp * 4);
  c->RG0.alloc(32L * 4 * c->H * 4);
  c->RG1.alloc(32L * 4 * c->H * 4);
  c->GS0.alloc(32L * 4 * c->H * 4);
  c->PS.alloc(32L * c->NPF * 4);
  c->ssum.alloc(32 * 4);
  c->pre1.alloc(32L * c->P * 4);
  c->pcnt.alloc(64 * 4);
  TT2_HIP(hipMemset(c->GS0.p, 0, c->GS0.bytes));  // rows >= B stay zero
  TT2_HIP(hipMemset(c->PS.p, 0, c->PS.bytes));
  c->c1.alloc(32L * c->H * 4);
  c->c2.alloc(32L * c->H * 4);
  c->Qp.alloc((long)c->KSQ * 32 * c->A * 4);
  c->energy.alloc(B * T * 4);
  c->cum.alloc(B * T * 4);
  c->max_att.alloc(64 * 4);
  c->PP.alloc((long)c->KSP * 32 * c->NPF * 4);
  c->ctl.alloc(sizeof(DecCtl));
  const long MF = MI * c->R;  // frame capacity: r frames per decoder step
  c->frames.alloc(B * MF * c->nm * 4);
  c->stop.alloc(B * MF * 4);
  c->align.alloc(B * T * MI * 4);
  c->dec.alloc(B * MF * c->nm * 4);
  c->post_a.alloc(B * MF * std::max(c->PC, c->nm) * 4);
  c->post_b.alloc(B * MF * std::max(c->PC, c->nm) * 4);
  c->mel.alloc(B * MF * c->nm * 4);
  {  // conv_x3 Postnet: TT2_POSTNET_CX=0 selects the im2col GEMMs
    const char* e = std::getenv("TT2_POSTNET_CX");
    c->post_cx = (!e || std::atoi(e) != 0) && c->PC % CX_BN == 0 && (cfg.postnet_kernel_size & 1) &&
                 cfg.postnet_kernel_size <= 2 * CX_P + 1;
  }
  {  // conv_x3 text encoder: TT2_ENC_CX=0 selects the im2col GEMMs
    const char* e = std::getenv("TT2_ENC_CX");
    c->enc_cx = (!e || std::atoi(e) != 0) && c->Cenc % CX_BN == 0 && c->E % 32 == 0 && (8 * c->U) % 4 == 0 &&
                (cfg.enc_conv_kernel_size & 1) && cfg.enc_conv_kernel_size <= 2 * CX_P + 1;
  }
  if (c->enc_cx) {
    const long rows = cx_rows((int)B, (int)T), w = std::max(c->E, c->Cenc);
    for (int i = 0; i < 2; ++i) {
      c->ex_h[i].alloc(rows * w * 2);
      c->ex_l[i].alloc(rows * w * 2);
    }
    c->ex_part.alloc((size_t)kEncSplitK * B * (T + 2 * CX_P) * c->Cenc * 4);
  }
  if (c->post_cx) {
    const long rows = cx_rows((int)B, (int)MF), cp0 = (c->nm + 31) / 32 * 32;
    c->px_in_h.alloc(rows * cp0 * 2);
    c->px_in_l.alloc(rows * cp0 * 2);
    for (int i = 0; i < 2; ++i) {
      c->px_h[i].alloc(rows * c->PC * 2);
      c->px_l[i].alloc(rows * c->PC * 2);
    }
  }
  TT2_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->ctl_host), 4 * sizeof(int)));
}

// ---------------------------------------------------------------- encode
static void encode_dev(tt2_ctx* c, const int* ids_d, const int* lens_d, const int* lens_h, int B, int T,
                       const float* ref_d[2], const int T_ref[2], hipStream_t s) {
  const auto& cfg = c->cfg;
  TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_finalize_weights not called");
  TT2_CHECK(B >= 1 && B <= cfg.max_batch && B <= 32, TT2_ERR_SHAPE_MISMATCH, "batch exceeds capacity (<=32)");
  TT2_CHECK(T >= 1 && T <= cfg.max_T_in, TT2_ERR_SHAPE_MISMATCH, "T_in exceeds capacity");
  for (int b = 0; b < B; ++b)
    TT2_CHECK(lens_h[b] >= 1 && lens_h[b] <= T, TT2_ERR_INVALID_ARG, "input_lengths must be in [1, T_in]");
  const int BT = B * T;
  if (c->emt.on())  // emotion labels (style_tokens query), pinned by tt2_set_emt_labels
    TT2_HIP(hipMemcpyAsync(c->emt.labels.p, c->emt_labels.data(), sizeof(int) * 32, hipMemcpyHostToDevice, s));
  // fork: the reference encoders (GST) depend only on the reference mels -> own stream, joined
  // before k_memory; they fill the CUs the 128-work-group persistent BiLSTM leaves idle
  const hipStream_t sr = (c->nmel > 0 && c->ref_stream) ? c->ref_stream : s;
  if (sr != s) {
    TT2_HIP(hipEventRecord(c->ref_ev[0], s));
    TT2_HIP(hipStreamWaitEvent(sr, c->ref_ev[0], 0));
  }
  hipLaunchKernelGGL(k_embed, dim3(BT), dim3(128), 0, s, ids_d, c->emb.as<float>(), c->x_a.as<float>(), BT, c->E,
                     cfg.n_symbols);
  TT2_HIP(hipGetLastError());
  // encoder convolutions: relu inside conv, then BN (modules.py:485-497, bnorm='after')
  if (c->enc_cx) {  // padded split planes, K split kEncSplitK ways (6.4k rows fill 204 tiles only)
    split_rows(c->x_a.as<float>(), B, T, c->E, (long)T * c->E, c->ex_h[0].as<_Float16>(), c->ex_l[0].as<_Float16>(),
               c->E, s);
    int cp = c->E, cur = 0;
    for (int i = 0; i < cfg.enc_conv_num_layers; ++i) {
      ConvX3Args a;
      a.Ah = c->ex_h[cur].as<_Float16>(); a.Al = c->ex_l[cur].as<_Float16>(); a.Cp = cp;
      a.B = B; a.T = T; a.kw = cfg.enc_conv_kernel_size;
      a.Bh = c->enc_cw_s[i].hi.as<_Float16>(); a.Bl = c->enc_cw_s[i].lo.as<_Float16>(); a.ldbt = c->enc_cw_s[i].ldbt;
      a.N = c->Cenc; a.bias = c->enc_cb[i].as<float>(); a.act = ACT_RELU;
      a.bn_scale = c->enc_bs[i].as<float>(); a.bn_shift = c->enc_bh[i].as<float>();
      a.Oh = c->ex_h[cur ^ 1].as<_Float16>(); a.Ol = c->ex_l[cur ^ 1].as<_Float16>();
      a.ks = enc_split_k(); a.part = c->ex_part.as<float>(); a.part_floats = (long)(c->ex_part.bytes / 4);
      conv_x3(a, s);
      cur ^= 1;
      cp = c->Cenc;
    }
    ConvX3Args a;  // BiLSTM input projection x·Wx + b for both directions: a width-1 conv -> xproj rows
    a.Ah = c->ex_h[cur].as<_Float16>(); a.Al = c->ex_l[cur].as<_Float16>(); a.Cp = cp; a.B = B; a.T = T; a.kw = 1;
    a.Bh = c->enc_wx_s.hi.as<_Float16>(); a.Bl = c->enc_wx_s.lo.as<_Float16>(); a.ldbt = c->enc_wx_s.ldbt;
    a.N = 8 * c->U; a.bias = c->enc_bx.as<float>(); a.Cout = c->xproj.as<float>(); a.ldc = 8 * c->U;
    conv_x3(a, s);
  } else {
  float* xin = c->x_a.as<float>();
  float* xout = c->x_b.as<float>();
  int cin = c->E;
  for (int i = 0; i < cfg.enc_conv_num_layers; ++i) {
    GemmArgs g;
    g.M = BT; g.N = c->Cenc; g.K = cfg.enc_conv_kernel_size * cin;
    g.a_mode = A_CONV1D; g.A = xin; g.T = T; g.C = cin; g.kw = cfg.enc_conv_kernel_size;
    g.pad = (cfg.enc_conv_kernel_size - 1) / 2; g.xs_b = (long)T * cin; g.xs_t = cin;
    g.Bw = c->enc_cw[i].as<float>(); g.ldb = c->Cenc; g.Cout = xout; g.ldc = c->Cenc;
    c->enc_cw_s[i].set(g);
    g.bias = c->enc_cb[i].as<float>(); g.act = ACT_RELU;
    g.bn_scale = c->enc_bs[i].as<float>(); g.bn_shift = c->enc_bh[i].as<float>();
    g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
    gemm(g, s);
    std::swap(xin, xout);
    cin = c->Cenc;
  }
  // BiLSTM: x·Wx + b for all t and both directions in one GEMM, then T recurrent steps
  {
    GemmArgs g;
    g.M = BT; g.N = 8 * c->U; g.K = cin; g.A = xin; g.lda = cin;
    g.Bw = c->enc_wx.as<float>(); g.ldb = 8 * c->U; g.Cout = c->xproj.as<float>(); g.ldc = 8 * c->U;
    g.bias = c->enc_bx.as<float>();
    g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
    gemm(g, s);
  }
  }
  zero_many({{c->enc_h.p, c->enc_h.bytes}, {c->enc_c.p, c->enc_c.bytes}, {c->enc_out.p, (size_t)BT * 2 * c->U * 4}}, s);
  int Tmax = 0;
  for (int b = 0; b < B; ++b) Tmax = std::max(Tmax, lens_h[b]);
  if (c->U == ENC_U && c->pd_dev_ok && c->pd_mode == 1 && c->kg_wmax_enc < KG_BMAX) {  // persistent (128 WGs)
    c->enc_hg.alloc(sizeof(unsigned long long) * 2 * 2 * 32 * ENC_U + 64);
    TT2_HIP(hipMemsetAsync(c->enc_hg.p, 0, c->enc_hg.bytes, s));
    EncPArgs a;
    a.xproj = c->xproj.as<float>(); a.wh = c->enc_wh.as<float>(); a.Hg = c->enc_hg.as<unsigned long long>();
    a.out = c->enc_out.as<float>(); a.lengths = lens_d; a.B = B; a.T = T; a.Tmax = Tmax;
    a.zo = cfg.zoneout; a.one_m_zo = (float)(1.0 - (double)cfg.zoneout);
    a.err = reinterpret_cast<int*>(a.Hg + 2 * 2 * 32 * ENC_U);
    {
      const char* e = std::getenv("TT2_ENC_SENTINEL");
      a.sentinel = e ? std::atoi(e) : 1;
    }
    void* params[] = {&a};  // cooperative: all 128 work-groups co-resident (h hand-offs spin)
    TT2_HIP(launch_persistent(reinterpret_cast<const void*>(k_enc_bilstm_persist), dim3(2 * ENC_U / 4),
                                       dim3(256), params, 0u, s));
    TT2_HIP(hipMemcpyAsync(&c->ctl_host[2], a.err, sizeof(int), hipMemcpyDeviceToHost, s));
    c->enc_err_check = true;
  } else
  for (int t = 0; t < Tmax; ++t) {
    EncLstmArgs a;
    a.xproj = c->xproj.as<float>(); a.wh = c->enc_wh.as<float>(); a.hs = c->enc_h.as<float>();
    a.cs = c->enc_c.as<float>(); a.out = c->enc_out.as<float>(); a.lengths = lens_d;
    a.B = B; a.T = T; a.U = c->U; a.t = t; a.zo = cfg.zoneout; a.one_m_zo = (float)(1.0 - (double)cfg.zoneout);
    hipLaunchKernelGGL(k_enc_lstm_step, dim3(2 * c->U / 4), dim3(256), 0, s, a);
  }
  TT2_HIP(hipGetLastError());
  // reference encoders + GST
  {
    const bool adain = c->style_mode == 2;
    float* bufs[2] = {c->conv_a.as<float>(), c->conv_b.as<float>()};
    // conv2d 3x3 'same' stack of reference encoder R over mel [B][TR][nm] (conv2d(), modules.py:
    // 499-511: conv, BN, ReLU; AdaIN: conv + ReLU, no BN, modules.py:84-87); NHWC out [B][H][W][C]
    auto conv_stack = [&](const RefNetDev& R, const float* x, int TR, int& H, int& Wd, int& C) -> float* {
      TT2_CHECK(TR >= 1 && TR <= cfg.max_T_ref, TT2_ERR_SHAPE_MISMATCH, "T_ref exceeds capacity");
      H = TR; Wd = c->nm; C = 1;
      float* out = nullptr;
      for (int i = 0; i < 6; ++i) {
        const int f = cfg.reference_filters[i], st = refnet_stride(adain, i);
        const int Ho = (H + st - 1) / st, Wo = (Wd + st - 1) / st;
        GemmArgs g;
        g.M = B * Ho * Wo; g.N = f; g.K = 9 * C; g.a_mode = A_CONV2D; g.A = x;
        g.H = H; g.Wd = Wd; g.C = C; g.Ho = Ho; g.Wo = Wo; g.kh = 3; g.kw2 = 3; g.sh = st; g.sw = st;
        g.pt = std::max((Ho - 1) * st + 3 - H, 0) / 2; g.pl = std::max((Wo - 1) * st + 3 - Wd, 0) / 2;
        g.Bw = R.cw[i].as<float>(); g.ldb = f; g.Cout = bufs[i & 1]; g.ldc = f;
        g.bias = R.cb[i].as<float>();
        if (adain) {
          g.act = ACT_RELU;
        } else {
          g.act = ACT_BN_RELU;
          g.bn_scale = R.bs[i].as<float>(); g.bn_shift = R.bh[i].as<float>();
        }
        g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
        g.kpart = c->kpart.as<float>(); g.kpart_floats = (long)(c->kpart.bytes / sizeof(float));  // deep layers: few tiles
        gemm(g, sr);
        x = out = bufs[i & 1];
        H = Ho; Wd = Wo; C = f;
      }
      return out;
    };
    // GRU over every frame + dense(128, tanh) (modules.py:57-64), then GST (gst=true) or the
    // embedding itself into the style columns [style_off, +128)
    auto gru_head = [&](const RefNetDev& R, const float* x, int H, int r, bool gst, float* style, int style_off) {
      const int D = cfg.reference_depth;
      c->refxg.alloc(sizeof(float) * (size_t)B * H * 3 * D);
      {  // x rows of the GRU gates + candidate kernels for every frame at once
        GemmArgs g;
        g.M = B * H; g.N = 3 * D; g.K = R.gin; g.A = x; g.lda = R.gin;
        g.Bw = R.wx.as<float>(); g.ldb = 3 * D; g.Cout = c->refxg.as<float>(); g.ldc = 3 * D;
        g.bias = R.bx.as<float>();
        g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
        g.kpart = c->kpart.as<float>(); g.kpart_floats = (long)(c->kpart.bytes / sizeof(float));
        gemm(g, sr);
      }
      RefGstArgs a;
      a.xg = c->refxg.as<float>(); a.T2 = H; a.D = D;
      a.whg = R.whg.as<float>(); a.whc = R.whc.as<float>();
      a.kd = R.kd.as<float>(); a.bd = R.bd.as<float>();
      a.tokens = gst ? R.tok.as<float>() : nullptr;
      a.kq = R.kq.as<float>(); a.bq = R.bq.as<float>(); a.kk = R.kk.as<float>(); a.bk = R.bk.as<float>();
      a.av = R.av.as<float>(); a.ag = R.ag.as<float>(); a.ab = R.ab.as<float>();
      a.ntok = cfg.num_gst; a.tokd = cfg.style_embed_depth / cfg.num_heads; a.A = cfg.style_att_dim;
      a.heads = cfg.num_heads; a.ref_out = c->ref_out.as<float>() + r * cfg.max_batch * 128;
      a.style = style; a.style_w = c->SW; a.style_off = style_off;
      const size_t shm = sizeof(float) * (a.D + a.D + 2 * a.D + 128 + a.A + a.ntok * a.A + a.ntok * a.tokd +
                                          a.heads * a.ntok + 16);
      hipLaunchKernelGGL(k_ref_gru_gst, dim3(B), dim3(256), shm, sr, a);
      TT2_HIP(hipGetLastError());
    };
    int H = 0, Wd = 0, C = 0;
    if (adain && !c->emt.on()) {
      // ReferenceEncoderAdaIn(spk, emt) (modules.py:75-107): the emotion map's per-channel moments
      // restyle the speaker map, which alone goes through the GRU (tacotron.py:242, 266-268)
      const RefNetDev& R = c->ref[0];
      float* mv_e = c->adain_mv.as<float>();
      float* mv_s = mv_e + (size_t)cfg.max_batch * cfg.reference_filters[5] * 2;
      float* xe = conv_stack(c->ref[1], ref_d[0], T_ref[0], H, Wd, C);  // emotion stack (conv2d_1 weights)
      hipLaunchKernelGGL(k_adain_moments, dim3(B, C), dim3(256), 0, sr, xe, H * Wd, C, mv_e);
      float* xs = conv_stack(R, ref_d[1], T_ref[1], H, Wd, C);
      hipLaunchKernelGGL(k_adain_moments, dim3(B, C), dim3(256), 0, sr, xs, H * Wd, C, mv_s);
      const long n = (long)B * H * Wd * C;
      hipLaunchKernelGGL(k_adain_mix, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, sr, xs, n, H * Wd, C, mv_s,
                         mv_e);
      TT2_HIP(hipGetLastError());
      TT2_CHECK(Wd * C == R.gin, TT2_ERR_SHAPE_MISMATCH, "reference encoder: GRU input width mismatch");
      gru_head(R, xs, H, 0, false, c->style.as<float>(), 0);
    } else {
      for (int r = 0; r < c->nref; ++r) {
        const RefNetDev& R = c->ref[r];
        const float* x = conv_stack(R, ref_d[r], T_ref[r], H, Wd, C);
        TT2_CHECK(Wd * C == R.gin, TT2_ERR_SHAPE_MISMATCH, "reference encoder: GRU input width mismatch");
        if (c->emt.on()) {
          if (r == 0) emt_encode(c->emt, x, B, H, sr);  // all_outputs=True: the attended values
          else gru_head(R, x, H, r, false, nullptr, 0);   // refnet_spk: the LSTM-1 speaker term
          continue;
        }
        const bool gst = c->style_mode == 0;
        gru_head(R, x, H, r, gst, c->style.as<float>(), r * (gst ? cfg.style_embed_depth : 128));
      }
    }
  }
  if (c->emt.attn == EMT_STYLE_TOKENS) emt_encode(c->emt, nullptr, B, 0, sr);
  if (sr != s) {  // join
    TT2_HIP(hipEventRecord(c->ref_ev[1], sr));
    TT2_HIP(hipStreamWaitEvent(s, c->ref_ev[1], 0));
  }
  hipLaunchKernelGGL(k_memory, dim3(BT), dim3(256), 0, s, c->enc_out.as<float>(), c->style.as<float>(), lens_d,
                     c->values.as<float>(), B, T, 2 * c->U, c->SW);
  TT2_HIP(hipGetLastError());
  {
    GemmArgs g;
    g.M = BT; g.N = c->A; g.K = c->Dm; g.A = c->values.as<float>(); g.lda = c->Dm;
    g.Bw = c->mem_k.as<float>(); g.ldb = c->A; g.Cout = c->keys.as<float>(); g.ldc = c->A;
    c->mem_k_s.set(g);
    g.kpart = c->kpart.as<float>(); g.kpart_floats = (long)(c->kpart.bytes / sizeof(float));
    g.bias = c->keys_b.as<float>();  // b_a + b_conv·W_loc (folded location-feature bias)
    g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
    gemm(g, s);
  }
  if (c->SW) {  // per-utterance style terms of the decoder: GS = style·W_lstm1[style rows], PS = style·W_proj[style rows]
    GemmArgs g;
    g.M = B; g.N = 4 * c->H; g.K = c->SW; g.A = c->style.as<float>(); g.lda = c->SW;
    g.Bw = c->l1_ws.as<float>(); g.ldb = 4 * c->H; g.Cout = c->GS0.as<float>(); g.ldc = 4 * c->H;
    g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
    g.kpart = c->kpart.as<float>(); g.kpart_floats = (long)(c->kpart.bytes / sizeof(float));
    gemm(g, s);
    GemmArgs p;
    p.M = B; p.N = c->NPF; p.K = c->SW; p.A = c->style.as<float>(); p.lda = c->SW;
    p.Bw = c->proj_ws.as<float>(); p.ldb = c->NPF; p.Cout = c->PS.as<float>(); p.ldc = c->NPF;
    p.split16 = 1;
    p.kpart = c->kpart.as<float>(); p.kpart_floats = (long)(c->kpart.bytes / sizeof(float));
    gemm(p, s);
  }
  if (c->l1_wspk.p && c->emt.spk) {  // emt 'simple': refnet_spk·W_lstm1[speaker rows] per utterance
    if (!c->SPK1.p) c->SPK1.alloc(32L * 4 * c->H * 4);
    // every encode: rows >= B must be zero (the persistent decoder folds all 32 rows into its
    // constants), also after an earlier encode of a larger batch
    TT2_HIP(hipMemsetAsync(c->SPK1.p, 0, c->SPK1.bytes, s));
    GemmArgs g;
    g.M = B; g.N = 4 * c->H; g.K = EMT_OUT; g.A = c->ref_out.as<float>() + (size_t)c->cfg.max_batch * 128; g.lda = EMT_OUT;
    g.Bw = c->l1_wspk.as<float>(); g.ldb = 4 * c->H; g.Cout = c->SPK1.as<float>(); g.ldc = 4 * c->H;
    g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
    g.kpart = c->kpart.as<float>(); g.kpart_floats = (long)(c->kpart.bytes / sizeof(float));
    gemm(g, s);
  }
  c->B = B;
  c->T_in = T;
  c->encoded = true;
  c->decoded = false;
}

// ---------------------------------------------------------------- decode
static long long* g_stamps_dev = nullptr;  // diagnostic s_memtime stamps (profiling only)
static long long* g_pd_stamps_dev = nullptr;  // [PD_NB][16] persistent-decoder stage stamps

static DecArgs make_dec_args(tt2_ctx* c, int max_iters, const uint8_t* masks_d, uint64_t seed,
                             const float* targets_d, int T_lim, float* frames_d, float* stop_d, float* align_d) {
  const auto& cfg = c->cfg;
  DecArgs a;
  a.ctl = c->ctl.as<DecCtl>();
  a.B = c->B; a.T_in = c->T_in; a.max_iters = max_iters; a.T_lim = targets_d ? T_lim : 0;
  a.nm = c->nm; a.P = c->P; a.H = c->H; a.Dm = c->Dm; a.E2 = c->E2; a.A = c->A; a.F = c->F; a.KL = c->KL;
  a.K1 = c->K1; a.Kp = c->Kp;
  a.zo = cfg.zoneout; a.one_m_zo = (float)(1.0 - (double)cfg.zoneout);
  a.stop_at_any = cfg.stop_at_any; a.mask_encoder = cfg.mask_encoder; a.cumulative = cfg.cumulative_weights;
  a.constraint = cfg.synthesis_constraint; a.monotonic = cfg.constraint_monotonic; a.win = cfg.attention_win_size;
  a.smoothing = cfg.smoothing;
  a.pre_b1 = c->pre_b1.as<float>();
  a.pre_w2 = c->pre_w2.as<float>(); a.pre_b2 = c->pre_b2.as<float>();
  a.KLp = c->KLp; a.Fp = c->Fp;
  a.q_w = c->q_w.as<float>(); a.loc_cw = c->loc_cw.as<float>(); a.va = c->va.as<float>();
  a.proj_w = c->proj_w.as<float>(); a.proj_b = c->proj_b.as<float>(); a.PS = c->PS.as<float>();
  a.keys = c->keys.as<float>(); a.values = c->values.as<float>(); a.lengths = c->lens.as<int>();
  for (int p = 0; p < 2; ++p) a.X1[p] = c->X1[p].as<float>();
  a.Xp = c->Xp.as<float>(); a.ssum = c->ssum.as<float>();
  a.Qp = c->Qp.as<float>(); a.energy = c->energy.as<float>(); a.cum = c->cum.as<float>();
  a.max_att = c->max_att.as<int>(); a.PP = c->PP.as<float>();
  a.KSQ = c->KSQ; a.KSP = c->KSP; a.NPJ = c->NPJ; a.NPF = c->NPF;
  a.TP1 = targets_d ? c->TP1.as<float>() : nullptr;
  a.pre1 = c->pre1.as<float>();
  a.masks = masks_d; a.seed = seed; a.targets = targets_d; a.stamps = nullptr;
  a.stamp_step = -1;
  if (const char* st = getenv("TT2_STAMP_STEP")) {  // diagnostic: prenet stamps of one decode step
    if (!g_stamps_dev) TT2_HIP(hipMalloc(&g_stamps_dev, 64 * sizeof(long long)));
    a.stamps = g_stamps_dev;
    a.stamp_step = atoi(st);
  }
  a.frames = frames_d; a.stop = stop_d; a.align = align_d;
  return a;
}

// refnet_spk output of the emt variant (null when it has none)
static const float* emt_spk(tt2_ctx* c) {
  return c->emt.spk ? c->ref_out.as<float>() + (size_t)c->cfg.max_batch * 128 : nullptr;
}

// The per-step launches (shared by the captured decode graph and the profiler).  `par` = step
// parity selecting the ping-pong state buffers.
static void launch_prenet(tt2_ctx* c, const DecArgs& a, int i, int t, hipStream_t s) {
  hipLaunchKernelGGL(k_prenet, dim3(c->P / 16), dim3(PRE_T), 0, s, a, i, t);
}
static LstmArgs lstm_args(tt2_ctx* c, const DecArgs& a, int layer, int par) {
  LstmArgs l;
  l.stamps = a.stamps;
  l.ctl = a.ctl; l.H = c->H; l.zo = a.zo; l.one_m_zo = a.one_m_zo; l.ho_off = 0;
  if (layer == 0) {
    l.X = a.X1[par]; l.K = c->K1; l.W = c->l1_w.as<float>(); l.b = c->l1_b.as<float>();
    l.RG = c->RG0.as<float>(); l.GS = c->GS0.as<float>(); l.ssum = c->ssum.as<float>();
    l.Hprev = c->H0s[par].as<float>(); l.Hz = c->H0s[par ^ 1].as<float>(); l.c = c->c1.as<float>();
    l.Xo = c->X2.as<float>();
  } else {
    l.X = c->X2.as<float>(); l.K = c->H; l.W = c->l2_w.as<float>(); l.b = c->l2_b.as<float>();
    l.RG = c->RG1.as<float>(); l.GS = nullptr; l.ssum = nullptr;
    l.Hprev = c->H1s[par].as<float>(); l.Hz = c->H1s[par ^ 1].as<float>(); l.c = c->c2.as<float>();
    l.Xo = c->Xp.as<float>();
  }
  return l;
}
static void launch_query(tt2_ctx* c, const DecArgs& a, const SideJob& sj, hipStream_t s) {
  PartArgs q;
  q.ctl = a.ctl; q.X = a.Xp; q.K = c->H; q.W = a.q_w; q.out = a.Qp; q.ldo = c->A; q.ntile = c->A / 16; q.KS = c->KSQ;
  launch_partial(q, sj, s);
}
static void launch_proj(tt2_ctx* c, const DecArgs& a, int t, const SideJob& sj, hipStream_t s) {
  ProjArgs p;
  // GTA feeds targets, not frames, to the prenet: the folded prenet-L1 columns are not needed
  p.ctl = a.ctl; p.X = a.Xp; p.K = c->Kp; p.W = a.proj_w; p.PP = a.PP; p.ldo = c->NPF;
  p.ntile = (a.targets ? c->NPJ : c->NPF) / 16;
  p.KS = c->KSP;
  p.cnt = c->pcnt.as<unsigned>();
  p.PS = a.PS; p.bias = a.proj_b; p.ssum = a.ssum; p.pre1 = c->pre1.as<float>();
  p.frames = a.frames; p.stop = a.stop;
  p.B = a.B; p.nm = a.nm; p.NPJ = c->NPJ; p.P = c->P; p.max_iters = a.max_iters; p.T_lim = a.T_lim;
  p.stop_at_any = a.stop_at_any; p.r = c->R; p.sc = c->SC;
  const int nsg = p.K / 16;
  const dim3 grid(p.ntile * p.KS + sj.ntile), blk(256);
  const int npw = nsg % (p.KS * 4) == 0 ? nsg / (p.KS * 4) : 0;
  if (npw == 6) hipLaunchKernelGGL(k_proj<6>, grid, blk, 0, s, p, sj, t);
  else if (npw == 4) hipLaunchKernelGGL(k_proj<4>, grid, blk, 0, s, p, sj, t);
  else if (npw == 8) hipLaunchKernelGGL(k_proj<8>, grid, blk, 0, s, p, sj, t);
  else if (npw == 2) hipLaunchKernelGGL(k_proj<2>, grid, blk, 0, s, p, sj, t);
  else hipLaunchKernelGGL(k_proj<0>, grid, blk, 0, s, p, sj, t);
}
// recurrent gate terms of step i+1 from the zoned states written at step i
static SideJob side_rec(tt2_ctx* c, int layer, int par) {
  SideJob j;
  j.X = (layer == 0 ? c->H0s[par ^ 1] : c->H1s[par ^ 1]).as<float>();
  j.W = (layer == 0 ? c->l1_wh : c->l2_wh).as<float>();
  j.out = (layer == 0 ? c->RG0 : c->RG1).as<float>();
  j.K = c->H;
  j.ntile = 4 * c->H / 16;
  j.delay = layer == 1 ? c->side_delay : c->side_delay2;  // RG1 runs in the energy launch, RG0 in softmax
  return j;
}
static void launch_energy(tt2_ctx* c, const DecArgs& a, const SideJob& sj, hipStream_t s) {
  const int nE = a.B * cdiv(a.T_in, 32);
  hipLaunchKernelGGL(k_energy, dim3(nE + sj.ntile), dim3(NWE * 64), 0, s, a, sj);
}
static void launch_softmax(tt2_ctx* c, const DecArgs& a, int i, int t, const SideJob& sj, hipStream_t s) {
  const size_t shm = sizeof(float) * std::max<size_t>(((a.T_in + 3) & ~3) + 4 * 16 * 16, 2048 + 512);
  hipLaunchKernelGGL(k_softmax_ctx, dim3(a.B * (c->E2 / 64) + sj.ntile), dim3(256), shm, s, a, i, t, sj);
}

static void launch_side(tt2_ctx* c, const DecArgs& a, const SideJob& sj, hipStream_t s) {
  hipLaunchKernelGGL(k_side, dim3(sj.ntile), dim3(256), 0, s, a.ctl, sj);
}

// side_mode 0: recurrent terms as extra blocks of the energy / softmax launches;
// side_mode 1: as launches on a second captured stream (parallel graph branches);
// side_mode 2: as extra blocks of the query / projection launches
static void enqueue_step(tt2_ctx* c, const DecArgs& a, int i, int t, hipStream_t s, hipStream_t s2) {
  const int par = i & 1;
  SideJob none = side_rec(c, 0, par);
  none.ntile = 0;
  launch_prenet(c, a, i, t, s);
  if (c->side_mode == 1 && i > 0) TT2_HIP(hipStreamWaitEvent(s, c->sev[2 * ((i - 1) & 1)], 0));
  launch_lstm(lstm_args(c, a, 0, par), c->H, s);
  if (c->side_mode == 1) {  // RG0 for step i+1 from h0(i)
    TT2_HIP(hipEventRecord(c->sev[4], s));
    TT2_HIP(hipStreamWaitEvent(s2, c->sev[4], 0));
    launch_side(c, a, side_rec(c, 0, par), s2);
    TT2_HIP(hipEventRecord(c->sev[2 * (i & 1)], s2));
  }
  if (c->side_mode == 1 && i > 0) TT2_HIP(hipStreamWaitEvent(s, c->sev[2 * ((i - 1) & 1) + 1], 0));
  launch_lstm(lstm_args(c, a, 1, par), c->H, s);
  if (c->emt.on())  // emotion context of step t -> LSTM-1 input block of step t+1
    emt_step_launch(c->emt, &a.ctl->done, a.Xp, a.X1[par ^ 1], c->P + c->E2, emt_spk(c), t, s);
  if (c->side_mode == 1) {  // RG1 for step i+1 from h1(i)
    TT2_HIP(hipEventRecord(c->sev[5], s));
    TT2_HIP(hipStreamWaitEvent(s2, c->sev[5], 0));
    launch_side(c, a, side_rec(c, 1, par), s2);
    TT2_HIP(hipEventRecord(c->sev[2 * (i & 1) + 1], s2));
  }
  launch_query(c, a, c->side_mode == 2 ? side_rec(c, 1, par) : none, s);
  launch_energy(c, a, c->side_mode == 0 ? side_rec(c, 1, par) : none, s);
  launch_softmax(c, a, i, t, c->side_mode == 0 ? side_rec(c, 0, par) : none, s);
  launch_proj(c, a, t, c->side_mode == 2 ? side_rec(c, 0, par) : none, s);
}

// ---- persistent decoder (decode_persist.hip) ----
// the persistent BiLSTM's timeout word, copied to host behind the launch; read after a sync
static void check_encoder(tt2_ctx* c) {
  if (!c->enc_err_check) return;
  c->enc_err_check = false;
  TT2_CHECK(c->ctl_host[2] == 0, TT2_ERR_HIP, "persistent BiLSTM encoder: a hand-off wait timed out");
}

// Tacotron_emt_attn decodes persistently in its 'multihead' form with the fork-default widths
// (query 128, heads x value width 512 or 1024, 2 x heads x attended rows <= 128, <= 32 dims per
// head); the other forms use the launch path
static bool pd_emt(const tt2_ctx* c) {
  const auto& m = c->emt;
  const int KC = m.heads * m.Dv;
  // 'multihead': contexts (KC = heads x Dv) -> attn_emt dense (128) = the block; 'style_tokens': 4 x 16
  // contexts over the 24 tokens = the 64-wide block (no dense, no refnet_spk term)
  const bool mh = m.attn == EMT_MULTIHEAD && m.XW == PD_EQ && (KC == 512 || KC == 1024) && c->pd_e_wd.p;
  const bool st = m.attn == EMT_STYLE_TOKENS && m.XW == 64 && KC == 64 && m.Dv == 16 && 2 * m.heads * m.Tv <= 192 &&
                  m.dh <= 32;
  // 'simple' (gru_multi at the fork widths): 128 units scored as 4 x 32-unit partials, one softmax per
  // row, the 128-wide context is the block's first half; the speaker half folds into the LSTM-1 bias
  const bool sp = m.attn == EMT_SIMPLE && m.Dv == PD_EQ && m.Tv <= 16 && (m.spk ? c->l1_wspk.p != nullptr : true) &&
                  m.XW == PD_EQ + (m.spk ? EMT_OUT : 0);
  return (mh || st || sp) && m.Aq == PD_EQ && m.Tv >= 1 && m.Tv <= 64 && c->K1 == PD_P + PD_E2 + m.XW;
}

static bool pd_fits(tt2_ctx* c) {
  return (!c->emt.on() || pd_emt(c)) && c->pd_mode == 1 && c->pd_dev_ok && c->kg_wmax_dec < KG_BMAX && c->H == PD_H && c->P == PD_P && c->E2 == PD_E2 && c->A == PD_A &&
         c->NPJ == PD_NPJ && c->NPF == PD_NPF && c->KLp == PD_KLP && c->T_in <= (c->emt.on() ? PD_TMAX : PD_TMAX_LONG) && c->B <= 32 &&
         !c->cfg.smoothing && c->R == 1;
}

static void decode_persist_dev(tt2_ctx* c, int max_iters, const uint8_t* masks_d, const float* targets_d, int T_lim,
                               float* frames_d, float* stop_d, float* align_d, hipStream_t s) {
  if (!c->H1x.p) {
    c->pd_ctl.alloc(sizeof(unsigned) * (2 * PD_NPH * PD_NB + 32 + 3 * PD_NREP * PD_NB));
    c->H1x.alloc(2L * 32 * PD_H * 4);
    c->H2x.alloc(2L * 32 * PD_H * 4);
    c->Ex.alloc(2L * 32 * 8 * PD_TMAX_LONG * 8);
    c->CTXx.alloc(2L * 32 * PD_E2 * 4);
    c->SSx.alloc(2L * 32 * 4);
    c->PPx.alloc(2L * PD_KSP * 32 * PD_NPF * 8);
    c->PREx.alloc(2L * 32 * PD_P * 8);
    for (auto& e : c->pd_ev) TT2_HIP(hipEventCreate(&e));
  }
  const bool emt = c->emt.on();
  if (emt && !c->QEx.p) {
    c->QEx.alloc(2L * PD_KSP * 32 * PD_EQ * 8);
    c->CMBx.alloc(2L * 32 * 1024 * 4);
    c->EOx.alloc(2L * PD_KSP * 32 * PD_EQ * 8);
    c->EMTx.alloc(2L * 32 * PD_EQ * 4);
  }
  const auto& cfg = c->cfg;
  // encoder steps the kernel covers: the values slice of 256 positions lives in registers; longer
  // inputs run the TM = 512 instance (the upper 256 positions streamed per step)
  const int tm = c->T_in > PD_TMAX ? PD_TMAX_LONG : PD_TMAX;
  c->keysT.alloc(sizeof(float) * (size_t)cfg.max_batch * PD_A * PD_TMAX_LONG);
  c->valuesT.alloc(sizeof(float) * (size_t)cfg.max_batch * PD_E2 * PD_TMAX_LONG);
  hipLaunchKernelGGL(k_transpose_bt, dim3(tm / 32, PD_A / 32, c->B), dim3(256), 0, s, c->keys.as<float>(),
                     (long)PD_A, c->keysT.as<float>(), c->T_in, PD_A, tm);
  hipLaunchKernelGGL(k_transpose_bt, dim3(tm / 32, PD_E2 / 32, c->B), dim3(256), 0, s, c->values.as<float>(),
                     (long)c->Dm, c->valuesT.as<float>(), c->T_in, PD_E2, tm);
  TT2_HIP(hipGetLastError());
  // flags + ctl words, every launch; granule tags restart at 1 every launch: a stale tag of an
  // earlier decode must never match.  The self-tagged h1 / h2 / context / Σ-align buffers are zeroed
  // too (tag bit 0, which steps 0 and 1 never expect: decode_persist.hip pd_tb)
  zero_many({{c->pd_ctl.p, c->pd_ctl.bytes}, {c->Ex.p, 2ul * 32 * 8 * tm * 8}, {c->PPx.p, c->PPx.bytes},
             {c->PREx.p, c->PREx.bytes}, {c->H1x.p, c->H1x.bytes}, {c->H2x.p, c->H2x.bytes},
             {c->CTXx.p, c->CTXx.bytes}, {c->SSx.p, c->SSx.bytes}}, s);
  if (emt) {
    zero_many({{c->QEx.p, c->QEx.bytes}, {c->EOx.p, c->EOx.bytes}, {c->EMTx.p, c->EMTx.bytes}}, s);
    // zero_state (Architecture_wrappers.py:182): the step-0 emotion block is refnet_spk alone
    const float* spk = c->emt.attn == EMT_MULTIHEAD ? emt_spk(c) : nullptr;  // 'multihead': spk is IN the block
    if (spk)
      hipLaunchKernelGGL(k_af_rows, dim3(c->B), dim3(PD_EQ), 0, s, spk, PD_EQ, c->EMTx.as<float>() + 32 * PD_EQ);
  }
  PdArgs a;
  a.flags = c->pd_ctl.as<unsigned>();
  a.flags2 = a.flags + PD_NPH * PD_NB;
  a.ctl = reinterpret_cast<int*>(a.flags + 2 * PD_NPH * PD_NB);
  a.rflags = a.flags + 2 * PD_NPH * PD_NB + 32;
  a.B = c->B; a.T_in = c->T_in; a.max_iters = max_iters; a.T_lim = targets_d ? T_lim : 0; a.nm = c->nm;
  a.stop_at_any = cfg.stop_at_any; a.mask_encoder = cfg.mask_encoder; a.cumulative = cfg.cumulative_weights;
  a.constraint = cfg.synthesis_constraint; a.monotonic = cfg.constraint_monotonic; a.win = cfg.attention_win_size;
  a.zo = cfg.zoneout; a.one_m_zo = (float)(1.0 - (double)cfg.zoneout);
  a.poll_sleep = 4;
  if (const char* e = getenv("TT2_PD_SLEEP")) a.poll_sleep = atoi(e);
  a.l1_w = c->pd_l1_w.as<float>(); a.l1_wh = c->pd_l1_wh.as<float>(); a.l1_b = c->l1_b.as<float>();  // x KG_SB
  a.l2_w = c->pd_l2_w.as<float>(); a.l2_wh = c->pd_l2_wh.as<float>(); a.l2_b = c->l2_b.as<float>();
  a.GS = c->GS0.as<float>(); a.q_wt = c->q_wt.as<float>(); a.loc_cw = c->loc_cw.as<float>(); a.va = c->va.as<float>();
  a.proj_w = c->pd_proj_w.as<float>(); a.proj_b = c->proj_b.as<float>(); a.PS = c->PS.as<float>();
  a.pre_b1 = c->pre_b1.as<float>(); a.pre_w2t = c->pre_w2t.as<float>(); a.pre_b2 = c->pre_b2.as<float>();
  a.TP1 = targets_d ? c->TP1.as<float>() : nullptr;
  a.keysT = c->keysT.as<float>(); a.valuesT = c->valuesT.as<float>(); a.lengths = c->lens.as<int>();
  a.masks = masks_d;
  a.H1x = c->H1x.as<float>(); a.H2x = c->H2x.as<float>(); a.Eg = c->Ex.as<unsigned long long>(); a.CTXx = c->CTXx.as<float>();
  a.SSx = c->SSx.as<float>(); a.PPg = c->PPx.as<unsigned long long>(); a.PREg = c->PREx.as<unsigned long long>();
  a.frames = frames_d; a.stop = stop_d;
  // alignments are written step-major (one contiguous T_in row per step and row: whole-line stores
  // instead of T_in scattered ones, which the CTX drain of the step waited for) and transposed to the
  // reference layout after the loop
  a.align = nullptr;
  if (align_d) {
    c->pd_alnT.alloc(sizeof(float) * (size_t)c->B * max_iters * c->T_in);
    a.align = c->pd_alnT.as<float>();
  }
  a.K1 = c->K1;
  if (emt) {
    const auto& m = c->emt;
    a.e_Tv = m.Tv; a.e_Dv = m.Dv; a.e_KC = m.heads * m.Dv; a.e_heads = m.heads; a.e_dh = m.dh;
    a.e_dense = m.attn == EMT_MULTIHEAD; a.e_XW = m.XW; a.e_vbs = m.val_bstride(); a.e_kbs = m.ke_bstride();
    a.e_simple = m.attn == EMT_SIMPLE;
    a.e_spk1 = nullptr;
    if (a.e_simple) {  // 4 unit-slice partials of 32 per score, context = the block's ctx half (128)
      a.e_heads = 4; a.e_dh = PD_EQ / 4; a.e_KC = PD_EQ; a.e_XW = PD_EQ;
      a.e_ab = m.vv.as<float>();  // unused ('simple' has no attention_b)
      if (m.spk) a.e_spk1 = c->SPK1.as<float>();
    }
    a.e_ke = m.ke.as<float>(); a.e_val = m.val.as<float>(); a.e_qrow = m.qrow.as<float>();
    a.e_vv = m.vv.as<float>(); a.e_ab = m.ab.as<float>(); a.e_wd = c->pd_e_wd.as<float>(); a.e_bd = m.bd.as<float>();
    a.e_spk = emt_spk(c); a.e_hist = m.hist.as<float>();
    a.QEg = c->QEx.as<unsigned long long>(); a.CMBx = c->CMBx.as<float>(); a.EOg = c->EOx.as<unsigned long long>();
    a.EMTx = c->EMTx.as<float>();
  }
  a.stamps = nullptr;
  a.stamp_step = -1;
  if (const char* st = getenv("TT2_STAMP_STEP")) {  // diagnostic: stage stamps of one decode step
    if (!g_pd_stamps_dev) TT2_HIP(hipMalloc(&g_pd_stamps_dev, PD_NB * 32 * sizeof(long long)));
    TT2_HIP(hipMemsetAsync(g_pd_stamps_dev, 0, PD_NB * 32 * sizeof(long long), s));
    a.stamps = g_pd_stamps_dev;
    a.stamp_step = atoi(st);
  }
  TT2_HIP(hipEventRecord(c->pd_ev[0], s));
  pd_launch(a, s, emt, tm);
  TT2_HIP(hipEventRecord(c->pd_ev[1], s));
  int h[4];
  TT2_HIP(hipMemcpyAsync(h, a.ctl, sizeof(h), hipMemcpyDeviceToHost, s));
  TT2_HIP(hipStreamSynchronize(s));
  TT2_HIP(hipEventElapsedTime(&c->pd_kernel_ms, c->pd_ev[0], c->pd_ev[1]));
  check_encoder(c);
  TT2_CHECK(h[2] == 0, TT2_ERR_HIP,
            "persistent decoder: a hand-off wait timed out (phase " + std::to_string(h[2] - 1) +
                "); set TT2_DECODER=launch to use the per-step launch path");
  TT2_CHECK(h[0] == 1, TT2_ERR_STATE, "persistent decoder did not terminate");
  c->n_steps = h[1];
  if (align_d && h[1] > 0) {
    hipLaunchKernelGGL(k_align_t, dim3((unsigned)((h[1] + 31) / 32), (unsigned)((c->T_in + 31) / 32), (unsigned)c->B),
                       dim3(256), 0, s, c->pd_alnT.as<float>(), h[1], c->T_in, (long)max_iters, align_d, (long)max_iters);
    TT2_HIP(hipGetLastError());
  }
  c->last_max_iters = max_iters;
  c->last_pd = true;
  c->have_args = false;
  c->decoded = true;
}

static void decode_dev(tt2_ctx* c, int max_iters, const uint8_t* masks_d, uint64_t seed, const float* targets_d,
                       int T_lim, float* frames_d, float* stop_d, float* align_d, hipStream_t s) {
  TT2_CHECK(c->encoded, TT2_ERR_STATE, "tt2_decode called before tt2_encode");
  TT2_CHECK(max_iters >= 1 && max_iters <= c->cfg.max_iters, TT2_ERR_SHAPE_MISMATCH, "max_iters exceeds capacity");
  TT2_CHECK(!targets_d || T_lim >= 1, TT2_ERR_INVALID_ARG, "targets given with T_targets < 1");
  // zero decoder state (zero_state, Architecture_wrappers.py:158-195; _go_frames helpers.py:136)
  zero_many({{c->X1[0].p, c->X1[0].bytes}, {c->X1[1].p, c->X1[1].bytes}, {c->H0s[0].p, c->H0s[0].bytes},
             {c->H0s[1].p, c->H0s[1].bytes}, {c->H1s[0].p, c->H1s[0].bytes}, {c->H1s[1].p, c->H1s[1].bytes},
             {c->X2.p, c->X2.bytes}, {c->Xp.p, c->Xp.bytes}, {c->RG0.p, c->RG0.bytes}, {c->RG1.p, c->RG1.bytes},
             {c->ssum.p, c->ssum.bytes}, {c->pcnt.p, c->pcnt.bytes}, {c->c1.p, c->c1.bytes}, {c->c2.p, c->c2.bytes},
             {c->cum.p, c->cum.bytes}, {c->max_att.p, c->max_att.bytes}, {c->ctl.p, sizeof(DecCtl)}},
            s);
  emt_init_launch(c->emt, emt_spk(c), c->X1[0].as<float>(), c->X1[1].as<float>(), c->P + c->E2, s);
  if (!masks_d) {  // prenet dropout keep bits from the counter-based device RNG
    const long n = (long)max_iters * 2 * c->B * c->P;
    c->gmasks.alloc((size_t)n);
    hipLaunchKernelGGL(k_gen_masks, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0, s,
                       c->gmasks.as<uint8_t>(), n, seed);
    TT2_HIP(hipGetLastError());
    masks_d = c->gmasks.as<uint8_t>();
  }
  if (targets_d) {  // GTA: prenet layer-1 pre-activations of every teacher frame, TP1 = targets·W1 + b1
    // targets_d is [B][T_lim·r][nm]: step t is fed frame t·r + r - 1 (targets[:, r-1::r], helpers.py:78)
    c->TP1.alloc(sizeof(float) * (size_t)c->B * T_lim * c->P);
    GemmArgs g;
    g.M = c->B * T_lim; g.N = c->P; g.K = c->nm; g.A = targets_d + (size_t)(c->R - 1) * c->nm; g.lda = c->nm * c->R;
    g.Bw = c->pre_w1r.as<float>(); g.ldb = c->P; g.Cout = c->TP1.as<float>(); g.ldc = c->P;
    g.bias = c->pre_b1.as<float>();
    gemm(g, s);
  }
  if (pd_fits(c)) {
    decode_persist_dev(c, max_iters, masks_d, targets_d, T_lim, frames_d, stop_d, align_d, s);
    return;
  }
  c->last_pd = false;
  const DecArgs a = make_dec_args(c, max_iters, masks_d, seed, targets_d, T_lim, frames_d, stop_d, align_d);
  c->last_args = a;
  c->have_args = true;
  auto key = std::make_tuple(c->B, c->T_in, max_iters, T_lim, (const void*)masks_d, (const void*)targets_d, seed,
                             (const void*)frames_d, (const void*)stop_d, (const void*)align_d);
  if (c->graph.key != key) {
    for (auto g : c->graph.chunks)
      if (g) (void)hipGraphExecDestroy(g);
    c->graph.chunks.clear();
    c->graph.key = key;
  }
  // one captured graph per S-step chunk (step index baked into the kernel arguments),
  // instantiated on first use and replayed by later calls with the same shapes
  auto chunk_graph = [&](int ch) -> hipGraphExec_t {
    if ((int)c->graph.chunks.size() <= ch) c->graph.chunks.resize(ch + 1, nullptr);
    if (!c->graph.chunks[ch]) {
      hipStream_t cs, cs2;
      TT2_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
      TT2_HIP(hipStreamCreateWithFlags(&cs2, hipStreamNonBlocking));
      hipGraph_t gr;
      TT2_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
      if (c->side_mode == 1) {  // fork the side stream into the capture
        TT2_HIP(hipEventRecord(c->sev[6], cs));
        TT2_HIP(hipStreamWaitEvent(cs2, c->sev[6], 0));
      }
      for (int i = 0; i < tt2_ctx::S; ++i) enqueue_step(c, a, i, ch * tt2_ctx::S + i, cs, cs2);
      if (c->side_mode == 1) {  // join: the chunk's last side jobs before the next chunk
        TT2_HIP(hipEventRecord(c->sev[7], cs2));
        TT2_HIP(hipStreamWaitEvent(cs, c->sev[7], 0));
      }
      TT2_HIP(hipStreamEndCapture(cs, &gr));
      TT2_HIP(hipGraphInstantiate(&c->graph.chunks[ch], gr, nullptr, nullptr, 0));
      TT2_HIP(hipGraphDestroy(gr));
      TT2_HIP(hipStreamDestroy(cs));
      TT2_HIP(hipStreamDestroy(cs2));
    }
    return c->graph.chunks[ch];
  };
  // launch chunks; watch the device `done` flag one chunk behind so the GPU never idles
  const int max_chunks = (max_iters + 1 + tt2_ctx::S - 1) / tt2_ctx::S;
  hipEvent_t ev[2];
  TT2_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
  TT2_HIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
  for (int ch = 0; ch < max_chunks; ++ch) {
    TT2_HIP(hipGraphLaunch(chunk_graph(ch), s));
    TT2_HIP(hipMemcpyAsync(&c->ctl_host[ch & 1], &c->ctl.as<DecCtl>()->done, sizeof(int), hipMemcpyDeviceToHost, s));
    TT2_HIP(hipEventRecord(ev[ch & 1], s));
    if (ch >= 1) {
      TT2_HIP(hipEventSynchronize(ev[(ch - 1) & 1]));
      if (c->ctl_host[(ch - 1) & 1]) break;
    }
  }
  TT2_HIP(hipEventDestroy(ev[0]));
  TT2_HIP(hipEventDestroy(ev[1]));
  DecCtl h;
  TT2_HIP(hipMemcpyAsync(&h, c->ctl.p, sizeof(DecCtl), hipMemcpyDeviceToHost, s));
  TT2_HIP(hipStreamSynchronize(s));
  TT2_CHECK(h.done, TT2_ERR_STATE, "decoder did not terminate");
  c->n_steps = h.n_steps;
  c->last_max_iters = max_iters;
  c->decoded = true;
}

// ---------------------------------------------------------------- postnet
static void postnet_dev(tt2_ctx* c, const float* frames_d, long frames_bstride, int B, int T, float* dec_d,
                        float* mel_d, hipStream_t s) {
  const auto& cfg = c->cfg;
  const float lo = cfg.symmetric_mels ? -cfg.max_abs_value - cfg.lower_bound_decay : 0.f - cfg.lower_bound_decay;
  const float hi = cfg.max_abs_value;
  const long n = (long)B * T * c->nm;
  hipLaunchKernelGGL(k_clip_frames, dim3((unsigned)std::min<long>(cdiv((int)std::min<long>(n, 1L << 30), 256), 4096)),
                     dim3(256), 0, s, frames_d, frames_bstride, dec_d, B, T, c->nm, lo, hi, cfg.clip_outputs);
  TT2_HIP(hipGetLastError());
  if (c->post_cx) {  // padded split planes between the layers (gemm.h conv_x3)
    const int cp0 = (c->nm + 31) / 32 * 32;
    split_rows(dec_d, B, T, c->nm, (long)T * c->nm, c->px_in_h.as<_Float16>(), c->px_in_l.as<_Float16>(), cp0, s);
    const _Float16 *ih = c->px_in_h.as<_Float16>(), *il = c->px_in_l.as<_Float16>();
    int cp = cp0;
    for (int i = 0; i < cfg.postnet_num_layers; ++i) {
      const SplitB& w = i == 0 ? c->post_cx0_s : c->post_cw_s[i];
      ConvX3Args a;
      a.Ah = ih; a.Al = il; a.Cp = cp; a.B = B; a.T = T; a.kw = cfg.postnet_kernel_size;
      a.Bh = w.hi.as<_Float16>(); a.Bl = w.lo.as<_Float16>(); a.ldbt = w.ldbt; a.N = c->PC;
      a.bias = c->post_cb[i].as<float>(); a.act = (i < cfg.postnet_num_layers - 1) ? ACT_TANH : ACT_NONE;
      a.bn_scale = c->post_bs[i].as<float>(); a.bn_shift = c->post_bh[i].as<float>();
      a.Oh = c->px_h[i & 1].as<_Float16>(); a.Ol = c->px_l[i & 1].as<_Float16>();
      conv_x3(a, s);
      ih = a.Oh; il = a.Ol; cp = c->PC;
    }
    ConvX3Args a;  // projection = a width-1 conv over the last planes, + residual, clip
    a.Ah = ih; a.Al = il; a.Cp = cp; a.B = B; a.T = T; a.kw = 1;
    a.Bh = c->post_pw_s.hi.as<_Float16>(); a.Bl = c->post_pw_s.lo.as<_Float16>(); a.ldbt = c->post_pw_s.ldbt;
    a.N = c->nm; a.bias = c->post_pb.as<float>(); a.Cout = mel_d; a.ldc = c->nm;
    a.residual = dec_d; a.ldr = c->nm; a.clip = cfg.clip_outputs; a.clip_lo = lo; a.clip_hi = hi;
    conv_x3(a, s);
    return;
  }
  const float* xin = dec_d;
  float* bufs[2] = {c->post_a.as<float>(), c->post_b.as<float>()};
  int cin = c->nm;
  for (int i = 0; i < cfg.postnet_num_layers; ++i) {
    GemmArgs g;
    g.M = B * T; g.N = c->PC; g.K = cfg.postnet_kernel_size * cin; g.a_mode = A_CONV1D; g.A = xin;
    g.T = T; g.C = cin; g.kw = cfg.postnet_kernel_size; g.pad = (cfg.postnet_kernel_size - 1) / 2;
    g.xs_b = (long)T * cin; g.xs_t = cin;
    g.Bw = c->post_cw[i].as<float>(); g.ldb = c->PC; g.Cout = bufs[i & 1]; g.ldc = c->PC;
    c->post_cw_s[i].set(g);
    g.bias = c->post_cb[i].as<float>(); g.act = (i < cfg.postnet_num_layers - 1) ? ACT_TANH : ACT_NONE;
    g.bn_scale = c->post_bs[i].as<float>(); g.bn_shift = c->post_bh[i].as<float>();
    g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
    gemm(g, s);
    xin = bufs[i & 1];
    cin = c->PC;
  }
  GemmArgs g;
  g.M = B * T; g.N = c->nm; g.K = c->PC; g.A = xin; g.lda = c->PC;
  g.Bw = c->post_pw.as<float>(); g.ldb = c->nm; g.Cout = mel_d; g.ldc = c->nm; g.bias = c->post_pb.as<float>();
  c->post_pw_s.set(g);
  g.residual = dec_d; g.ldr = c->nm; g.clip = cfg.clip_outputs; g.clip_lo = lo; g.clip_hi = hi;
  g.split16 = 1;  // fp16x3 split MFMA (gemm.h): operands bounded, error ~1e-7 relative
  gemm(g, s);
}

}  // namespace tt2

using namespace tt2;

namespace tt2 {
// STREAM-like copy (confirm the HBM peak on the box next to the 8 TB/s spec):
// dst = src over two `bytes` buffers (>> the 256 MB MALL), 16-byte loads and stores; each
// work-group copies contiguous 256·U-float4 blocks with all U loads in flight before the stores
// (NT: non-temporal loads / stores).  Counted bytes = read + write.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_hbm_copy(const f32x4* __restrict__ src, f32x4* __restrict__ dst, long n4) {
  const long nblk = n4 / (256L * U);
  for (long blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const long base = blk * 256L * U + threadIdx.x;
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + base + 256L * u) : src[base + 256L * u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], dst + base + 256L * u);
      else dst[base + 256L * u] = v[u];
    }
  }
  for (long i = nblk * 256L * U + (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) dst[i] = src[i];
}

}  // namespace tt2

extern "C" {

const char* tt2_last_error(void) { return g_last_error.c_str(); }

static int g_exit_status = 1;
static void tt2_exit_guard_handler() {
  std::fflush(stdout);
  std::fflush(stderr);
  _exit(g_exit_status);
}
void tt2_exit_guard(int install, int status) {
  static bool installed = false;
  if (install && !installed) {
    std::atexit(tt2_exit_guard_handler);
    installed = true;
  }
  g_exit_status = status;
}
const char* tt2_version(void) { return "libtt2 0.1 gfx950 fp32 (MFMA f32)"; }

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
  c->predict_linear = 0; c->num_freq = 1025; c->cbhg_kernels = 8; c->cbhg_conv_channels = 128;
  c->cbhg_pool_size = 2; c->cbhg_projection = 256; c->cbhg_projection_kernel_size = 3;
  c->cbhg_highwaynet_layers = 4; c->cbhg_highway_units = 128; c->cbhg_rnn_units = 128;
  c->smoothing = 0; c->outputs_per_step = 1;
}

tt2_status tt2_create(const tt2_config* cfg, int hip_device, tt2_ctx** out) {
  return guard([&] {
    TT2_CHECK(cfg && out, TT2_ERR_INVALID_ARG, "tt2_create: null argument");
    *out = nullptr;
    int ndev = 0;
    TT2_HIP(hipGetDeviceCount(&ndev));
    TT2_CHECK(hip_device >= 0 && hip_device < ndev, TT2_ERR_INVALID_ARG, "tt2_create: bad device index");
    TT2_CHECK(cfg->max_batch >= 1 && cfg->max_batch <= 32, TT2_ERR_INVALID_ARG, "max_batch must be in [1, 32]");
    TT2_CHECK(cfg->max_T_in >= 1 && cfg->max_iters >= 1, TT2_ERR_INVALID_ARG, "capacities must be >= 1");
    TT2_CHECK(cfg->num_mels <= 80 && cfg->num_mels >= 1, TT2_ERR_INVALID_ARG, "num_mels must be <= 80");
    TT2_CHECK(cfg->prenet_units % 16 == 0 && cfg->prenet_units <= 256, TT2_ERR_INVALID_ARG,
              "prenet_units must be a multiple of 16, <= 256");
    TT2_CHECK(cfg->decoder_lstm_units % 16 == 0, TT2_ERR_INVALID_ARG, "decoder_lstm_units % 16 != 0");
    TT2_CHECK(cfg->encoder_lstm_units % 16 == 0, TT2_ERR_INVALID_ARG, "encoder_lstm_units % 16 != 0");
    TT2_CHECK(cfg->attention_dim % 16 == 0 && cfg->attention_dim >= 16, TT2_ERR_INVALID_ARG, "attention_dim % 16 != 0");
    TT2_CHECK(cfg->attention_kernel % 2 == 1, TT2_ERR_INVALID_ARG, "attention_kernel must be odd");
    auto c = std::make_unique<tt2_ctx>();
    c->cfg = *cfg;
    c->dev = hip_device;
    TT2_HIP(hipSetDevice(hip_device));
    TT2_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    TT2_HIP(hipStreamCreateWithFlags(&c->ref_stream, hipStreamNonBlocking));
    for (auto& e : c->ref_ev) TT2_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->nm = cfg->num_mels; c->E = cfg->embedding_dim; c->Cenc = cfg->enc_conv_channels; c->U = cfg->encoder_lstm_units;
    c->A = cfg->attention_dim; c->F = cfg->attention_filters; c->KL = cfg->attention_kernel; c->P = cfg->prenet_units;
    c->H = cfg->decoder_lstm_units; c->PC = cfg->postnet_channels;
    c->KLp = (c->KL + 15) / 16 * 16; c->Fp = (c->F + 15) / 16 * 16;
    TT2_CHECK(c->KLp <= 64 && c->Fp <= 64, TT2_ERR_INVALID_ARG, "attention_kernel / attention_filters must be <= 64");
    TT2_CHECK(c->A <= 256, TT2_ERR_INVALID_ARG, "attention_dim must be <= 256");
    const bool emt = cfg->emt_attn != EMT_OFF;
    if (emt) {
      // Tacotron_emt_attn: the attention memory is the encoder output alone (tacotron_emt_attn.py:
      // 244-246); refnet_emt feeds the emotion attention, refnet_spk the LSTM input; no GST
      c->nref = cfg->emt_attn == EMT_STYLE_TOKENS ? 0 : (cfg->emt_only ? 1 : 2);
      c->SW = 0;
    } else {
      // style path (tacotron.py:236-308): use_gst=False takes the reference embeddings themselves
      c->style_mode = (!cfg->use_gst && cfg->style_mode == 0) ? 1 : cfg->style_mode;
      TT2_CHECK(c->style_mode >= 0 && c->style_mode <= 2, TT2_ERR_INVALID_ARG, "style_mode must be 0..2");
      c->nref = c->style_mode == 2 ? 1 : (cfg->emt_only ? 1 : 2);
      TT2_CHECK(!(c->style_mode == 2 && cfg->emt_only), TT2_ERR_INVALID_ARG,
                "must provide speaker reference to use AdaIn");  // tacotron.py:60-61
      c->SW = c->style_mode == 0 ? c->nref * cfg->style_embed_depth : 128 * c->nref;
    }
    c->nmel = c->style_mode == 2 ? 2 : c->nref;
    c->Dm = 2 * c->U + c->SW;
    TT2_CHECK(c->Dm % 64 == 0, TT2_ERR_INVALID_ARG, "memory width must be a multiple of 64");
    c->E2 = 2 * c->U;
    emt_configure(c->emt, cfg->emt_attn, cfg->emt_ref_gru, cfg->emt_only, cfg->n_emt, c->H, c->A, cfg->style_att_dim,
                  cfg->num_heads, cfg->reference_depth, c->nm, cfg->reference_filters, cfg->max_batch,
                  cfg->max_T_ref, cfg->max_iters);
    c->emt_labels.assign(32, 0);
    // LSTM-1 critical rows: [prenet | context_enc | emotion block (emt variant)]
    c->K1 = c->P + c->E2 + c->emt.XW; c->Kp = c->H + c->E2;
    TT2_CHECK(c->E2 % 64 == 0, TT2_ERR_INVALID_ARG, "2*encoder_lstm_units must be a multiple of 64");
    // outputs_per_step r (tacotron.py:322-324): frame columns [0, nm·r), then the r stop columns from
    // SC inside ONE 16-column tile (the tile whose last arriver applies the stop rule)
    c->R = cfg->outputs_per_step;
    TT2_CHECK(c->R >= 1 && c->R <= 8, TT2_ERR_INVALID_ARG, "outputs_per_step must be in [1, 8]");
    c->SC = (c->nm * c->R) % 16 + c->R <= 16 ? c->nm * c->R : (c->nm * c->R + 15) / 16 * 16;
    c->NPJ = ((c->SC + c->R + 15) / 16) * 16;
    c->NPF = c->NPJ + c->P;
    alloc_acts(c.get());
    for (auto& e : c->ev) TT2_HIP(hipEventCreate(&e));
    for (auto& e : c->sev) TT2_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (const char* m = getenv("TT2_DECODER")) c->pd_mode = std::string(m) == "launch" ? 0 : 1;
    c->pd_dev_ok = pd_device_ok(hip_device);
    if (const char* m = getenv("TT2_SIDE_MODE")) c->side_mode = atoi(m);
    if (const char* m = getenv("TT2_SIDE_DELAY")) c->side_delay = atoi(m);
    if (const char* m = getenv("TT2_SIDE_DELAY2")) c->side_delay2 = atoi(m);
    *out = c.release();
  });
}

void tt2_destroy(tt2_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  for (auto g : c->graph.chunks)
    if (g) (void)hipGraphExecDestroy(g);
  if (c->ctl_host) (void)hipHostFree(c->ctl_host);
  for (auto& e : c->pd_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->sev)
    if (e) (void)hipEventDestroy(e);
  if (c->ref_stream) (void)hipStreamSynchronize(c->ref_stream);
  for (auto& e : c->ref_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->ref_stream) (void)hipStreamDestroy(c->ref_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;  // DevBuf destructors release the device buffers
}

tt2_status tt2_load_tensor(tt2_ctx* c, const char* name, const float* host, const int64_t* shape, int ndim) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    put_tensor(c->host, name, host, shape, ndim);
    c->finalized = false;
  });
}

tt2_status tt2_finalize_weights(tt2_ctx* c) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    finalize(c);
  });
}

tt2_status tt2_encode(tt2_ctx* c, const int32_t* ids, const int32_t* lengths, int B, int T_in, const float* ref_emt,
                      int T_ref_emt, const float* ref_spk, int T_ref_spk, float* memory_out, float* style_out) {
  return guard([&] {
    TT2_CHECK(c && ids && lengths, TT2_ERR_INVALID_ARG, "tt2_encode: null argument");
    TT2_CHECK(B >= 1 && B <= c->cfg.max_batch, TT2_ERR_SHAPE_MISMATCH, "batch exceeds capacity");
    TT2_CHECK(T_in >= 1 && T_in <= c->cfg.max_T_in, TT2_ERR_SHAPE_MISMATCH, "T_in exceeds capacity");
    TT2_CHECK(c->nmel == 0 || (ref_emt && (c->nmel < 2 || ref_spk)), TT2_ERR_INVALID_ARG,
              "must provide references");  // tacotron.py:66-67, tacotron_emt_attn.py:72-73
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    TT2_HIP(hipMemcpyAsync(c->ids.p, ids, sizeof(int) * B * T_in, hipMemcpyHostToDevice, s));
    TT2_HIP(hipMemcpyAsync(c->lens.p, lengths, sizeof(int) * B, hipMemcpyHostToDevice, s));
    const float* refs[2] = {ref_emt, ref_spk};
    const int trs[2] = {T_ref_emt, T_ref_spk};
    const float* ref_d[2] = {nullptr, nullptr};
    for (int r = 0; r < c->nmel; ++r) {
      TT2_CHECK(trs[r] >= 1 && trs[r] <= c->cfg.max_T_ref, TT2_ERR_SHAPE_MISMATCH, "T_ref exceeds capacity");
      TT2_HIP(hipMemcpyAsync(c->refm[r].p, refs[r], sizeof(float) * B * trs[r] * c->nm, hipMemcpyHostToDevice, s));
      ref_d[r] = c->refm[r].as<float>();
    }
    encode_dev(c, c->ids.as<int>(), c->lens.as<int>(), lengths, B, T_in, ref_d, trs, s);
    TT2_HIP(hipStreamSynchronize(s));
    check_encoder(c);
    if (memory_out)
      TT2_HIP(hipMemcpyAsync(memory_out, c->values.p, sizeof(float) * B * T_in * c->Dm, hipMemcpyDeviceToHost, s));
    if (style_out && c->SW)
      for (int b = 0; b < B; ++b)
        TT2_HIP(hipMemcpyAsync(style_out + (size_t)b * c->SW, c->style.as<float>() + (size_t)b * c->SW,
                               sizeof(float) * c->SW, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
  });
}

static void decoder_step_dev(tt2_ctx* c, const float* frame_in, const uint8_t* masks,
                             const tt2_decoder_state* in, tt2_decoder_state* out, float* frame_out, float* stop_out,
                             float* align_out) {
  TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_finalize_weights not called");
  TT2_CHECK(c->encoded, TT2_ERR_STATE, "tt2_decoder_step called before tt2_encode");
  TT2_CHECK(!c->emt.on(), TT2_ERR_INVALID_ARG,
            "tt2_decoder_step: the Tacotron_emt_attn variant decodes through tt2_decode / tt2_synthesize_dev");
  TT2_CHECK(c->R == 1, TT2_ERR_INVALID_ARG, "tt2_decoder_step: outputs_per_step > 1 decodes through tt2_decode");
  TT2_CHECK(frame_in && masks && in && out && frame_out && stop_out, TT2_ERR_INVALID_ARG,
            "tt2_decoder_step: null argument");
  TT2_CHECK(in->h1 && in->c1 && in->h2 && in->c2 && in->attention && in->alignments && in->max_attentions &&
                out->h1 && out->c1 && out->h2 && out->c2 && out->attention && out->alignments && out->max_attentions,
            TT2_ERR_INVALID_ARG, "tt2_decoder_step: null state array");
  const auto& cfg = c->cfg;
  const std::string P(TP);
  const WeightMap& wm = c->host;
  hipStream_t s = c->stream;
  if (!c->st_ready) {  // raw row-major variables, exactly as loaded
    const char* names[16] = {"decoder/decoder_prenet/dense_1/kernel", "decoder/decoder_prenet/dense_1/bias",
                             "decoder/decoder_prenet/dense_2/kernel", "decoder/decoder_prenet/dense_2/bias",
                             "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel",
                             "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/bias",
                             "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/kernel",
                             "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/bias", "decoder/query_layer/kernel",
                             "decoder/Location_Sensitive_Attention/location_features_convolution/kernel",
                             "decoder/Location_Sensitive_Attention/location_features_layer/kernel",
                             "decoder/Location_Sensitive_Attention/attention_variable_projection",
                             "decoder/linear_transform_projection/projection_linear_transform_projection/kernel",
                             "decoder/linear_transform_projection/projection_linear_transform_projection/bias",
                             "decoder/stop_token_projection/projection_stop_token_projection/kernel",
                             "decoder/stop_token_projection/projection_stop_token_projection/bias"};
    for (int i = 0; i < 16; ++i) {
      auto it = wm.find(P + names[i]);
      TT2_CHECK(it != wm.end(), TT2_ERR_NOT_LOADED, std::string("missing variable ") + P + names[i]);
      upload(c->st_w[i], it->second);
    }
    c->st_ready = true;
  }
  StepWeights w;
  const float* const* wp[16] = {&w.pre_w1, &w.pre_b1, &w.pre_w2, &w.pre_b2, &w.k1, &w.b1, &w.k2, &w.b2,
                                &w.wq, &w.wconv, &w.wloc, &w.va, &w.wf, &w.bf, &w.ws, &w.bs};
  for (int i = 0; i < 16; ++i) *const_cast<const float**>(wp[i]) = c->st_w[i].as<float>();
  StepDims d;
  d.B = c->B; d.T = c->T_in; d.nm = c->nm; d.P = c->P; d.H = c->H; d.D = c->Dm; d.A = c->A; d.F = c->F; d.KL = c->KL;
  d.zo = cfg.zoneout; d.cumulative = cfg.cumulative_weights; d.constraint = cfg.synthesis_constraint;
  d.monotonic = cfg.constraint_monotonic; d.win = cfg.attention_win_size; d.mask_encoder = cfg.mask_encoder;
  d.smoothing = cfg.smoothing;
  const size_t B = d.B, nH = B * d.H, nD = B * d.D, nT = B * d.T;
  // device image of [frame_in | 4 states | ctx | cum | max_att | masks] in and the outputs
  const size_t f_in = B * d.nm, n_in = f_in + 4 * nH + nD + nT, n_out = 4 * nH + nD + nT + f_in + B + nT;
  const size_t bytes = sizeof(float) * (n_in + n_out) + 2 * sizeof(int) * B + 2 * B * d.P + 64;
  c->st_io.alloc(bytes);
  c->st_scratch.alloc(sizeof(float) * step_scratch_floats(d));
  float* base = c->st_io.as<float>();
  float* fi = base;
  float* h1 = fi + f_in; float* c1 = h1 + nH; float* h2 = c1 + nH; float* c2 = h2 + nH;
  float* cx = c2 + nH; float* cu = cx + nD;
  float* o = cu + nT;
  float* h1o = o; float* c1o = h1o + nH; float* h2o = c1o + nH; float* c2o = h2o + nH;
  float* cxo = c2o + nH; float* cuo = cxo + nD; float* fo = cuo + nT; float* so = fo + f_in; float* ao = so + B;
  int* ma = reinterpret_cast<int*>(ao + nT);
  int* mao = ma + B;
  uint8_t* mk = reinterpret_cast<uint8_t*>(mao + B);
  auto h2d = [&](void* dst, const void* src, size_t n) { TT2_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s)); };
  auto d2h = [&](void* dst, const void* src, size_t n) { TT2_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s)); };
  h2d(fi, frame_in, 4 * f_in);
  h2d(h1, in->h1, 4 * nH); h2d(c1, in->c1, 4 * nH); h2d(h2, in->h2, 4 * nH); h2d(c2, in->c2, 4 * nH);
  h2d(cx, in->attention, 4 * nD); h2d(cu, in->alignments, 4 * nT); h2d(ma, in->max_attentions, 4 * B);
  h2d(mk, masks, 2 * B * d.P);
  StepIO io;
  io.keys = c->keys.as<float>(); io.values = c->values.as<float>(); io.lengths = c->lens.as<int>();
  io.frame_in = fi; io.masks = mk;
  io.h1 = h1; io.c1 = c1; io.h2 = h2; io.c2 = c2; io.ctx = cx; io.cum = cu; io.max_att = ma;
  io.h1o = h1o; io.c1o = c1o; io.h2o = h2o; io.c2o = c2o; io.ctxo = cxo; io.cumo = cuo; io.max_att_o = mao;
  io.frame = fo; io.stop = so; io.align = ao; io.scratch = c->st_scratch.as<float>();
  decoder_step_launch(w, d, io, s);
  d2h(out->h1, h1o, 4 * nH); d2h(out->c1, c1o, 4 * nH); d2h(out->h2, h2o, 4 * nH); d2h(out->c2, c2o, 4 * nH);
  d2h(out->attention, cxo, 4 * nD); d2h(out->alignments, cuo, 4 * nT); d2h(out->max_attentions, mao, 4 * B);
  d2h(frame_out, fo, 4 * f_in); d2h(stop_out, so, 4 * B);
  if (align_out) d2h(align_out, ao, 4 * nT);
  TT2_HIP(hipStreamSynchronize(s));
  out->time = in->time + 1;
}

tt2_status tt2_decoder_step(tt2_ctx* c, const float* frame_in, const uint8_t* prenet_masks,
                            const tt2_decoder_state* state_in, tt2_decoder_state* state_out, float* frame_out,
                            float* stop_out, float* alignments_out) {
  return guard([&] {
    TT2_CHECK(c, TT2_ERR_INVALID_ARG, "null ctx");
    TT2_HIP(hipSetDevice(c->dev));
    decoder_step_dev(c, frame_in, prenet_masks, state_in, state_out, frame_out, stop_out, alignments_out);
  });
}

tt2_status tt2_prenet_keep_bits(uint64_t seed, int max_iters, int B, int prenet_units, uint8_t* out) {
  return guard([&] {
    TT2_CHECK(out, TT2_ERR_INVALID_ARG, "tt2_prenet_keep_bits: null argument");
    TT2_CHECK(max_iters >= 1 && B >= 1 && prenet_units >= 1, TT2_ERR_INVALID_ARG, "tt2_prenet_keep_bits: bad sizes");
    const long n = (long)max_iters * 2 * B * prenet_units;
    DevBuf d;
    d.alloc((size_t)n);
    hipLaunchKernelGGL(k_gen_masks, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0, 0,
                       d.as<uint8_t>(), n, seed);
    TT2_HIP(hipGetLastError());
    TT2_HIP(hipMemcpy(out, d.p, (size_t)n, hipMemcpyDeviceToHost));
  });
}

tt2_status tt2_decode(tt2_ctx* c, int max_iters, const uint8_t* prenet_masks, uint64_t seed, const float* targets,
                      int T_targets, float* frames, float* stop, float* align, int32_t* n_steps) {
  return guard([&] {
    TT2_CHECK(c && frames && stop && n_steps, TT2_ERR_INVALID_ARG, "tt2_decode: null argument");
    TT2_CHECK(c->encoded, TT2_ERR_STATE, "tt2_decode called before tt2_encode");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    const int B = c->B;
    const uint8_t* masks_d = nullptr;
    if (prenet_masks) {
      const size_t n = (size_t)max_iters * 2 * B * c->P;
      c->masks.alloc(n);
      TT2_HIP(hipMemcpyAsync(c->masks.p, prenet_masks, n, hipMemcpyHostToDevice, s));
      masks_d = c->masks.as<uint8_t>();
    }
    const float* tg_d = nullptr;
    const int r = c->R;
    int T_lim = 0;
    if (targets) {
      TT2_CHECK(T_targets >= r, TT2_ERR_INVALID_ARG, "T_targets must be >= outputs_per_step");
      // TacoTrainingHelper runs len(targets[:, r-1::r]) = T_targets / r steps (helpers.py:78-81); the
      // device copy keeps the first T_lim·r frames of each row
      T_lim = T_targets / r;
      const size_t row = (size_t)T_lim * r * c->nm * sizeof(float);
      c->targets.alloc(row * B);
      TT2_HIP(hipMemcpy2DAsync(c->targets.p, row, targets, (size_t)T_targets * c->nm * sizeof(float), row, B,
                               hipMemcpyHostToDevice, s));
      tg_d = c->targets.as<float>();
    }
    decode_dev(c, max_iters, masks_d, seed, tg_d, T_lim, c->frames.as<float>(), c->stop.as<float>(),
               align ? c->align.as<float>() : nullptr, s);
    const int n = c->n_steps;
    *n_steps = n;
    const size_t fs = (size_t)max_iters * r;  // frames per row in the caller's and the device layout
    for (int b = 0; b < B; ++b) {
      TT2_HIP(hipMemcpyAsync(frames + b * fs * c->nm, c->frames.as<float>() + b * fs * c->nm,
                             sizeof(float) * n * r * c->nm, hipMemcpyDeviceToHost, s));
      TT2_HIP(hipMemcpyAsync(stop + b * fs, c->stop.as<float>() + b * fs, sizeof(float) * n * r,
                             hipMemcpyDeviceToHost, s));
    }
    if (align)
      TT2_HIP(hipMemcpyAsync(align, c->align.p, sizeof(float) * B * c->T_in * max_iters, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
  });
}

tt2_status tt2_postnet(tt2_ctx* c, const float* frames_in, int B, int T, float* decoder_output, float* mel_out) {
  return guard([&] {
    TT2_CHECK(c && mel_out, TT2_ERR_INVALID_ARG, "tt2_postnet: null argument");
    TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_finalize_weights not called");
    TT2_CHECK(B >= 1 && B <= c->cfg.max_batch && T >= 1 && T <= c->cfg.max_iters * c->R, TT2_ERR_SHAPE_MISMATCH,
              "postnet: shape exceeds capacity");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    const float* src;
    long bstride;
    if (frames_in) {
      // stage caller frames in post_a: the clip kernel moves them to `dec` before conv 1 reuses post_a
      TT2_CHECK((size_t)B * T * c->nm * 4 <= c->post_a.bytes, TT2_ERR_SHAPE_MISMATCH, "postnet staging too small");
      TT2_HIP(hipMemcpyAsync(c->post_a.p, frames_in, sizeof(float) * B * T * c->nm, hipMemcpyHostToDevice, s));
      src = c->post_a.as<float>();
      bstride = (long)T * c->nm;
    } else {
      TT2_CHECK(c->decoded, TT2_ERR_STATE, "tt2_postnet(NULL) called before tt2_decode");
      TT2_CHECK(B == c->B && T == c->n_steps * c->R, TT2_ERR_SHAPE_MISMATCH, "postnet shape differs from last decode");
      src = c->frames.as<float>();
      bstride = (long)c->last_max_iters * c->R * c->nm;
    }
    postnet_dev(c, src, bstride, B, T, c->dec.as<float>(), c->mel.as<float>(), s);
    if (decoder_output)
      TT2_HIP(hipMemcpyAsync(decoder_output, c->dec.p, sizeof(float) * B * T * c->nm, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipMemcpyAsync(mel_out, c->mel.p, sizeof(float) * B * T * c->nm, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
  });
}

tt2_status tt2_synthesize_dev(tt2_ctx* c, const int32_t* ids_d, const int32_t* lengths_d, const int32_t* lengths_host,
                              int B, int T_in, const float* ref_emt_d, int T_ref_emt, const float* ref_spk_d,
                              int T_ref_spk, int max_iters, const uint8_t* prenet_masks_d, uint64_t seed,
                              float* mel_d, float* stop_d, int32_t* n_steps_host, void* stream) {
  return guard([&] {
    TT2_CHECK(c && ids_d && lengths_d && lengths_host && mel_d && n_steps_host, TT2_ERR_INVALID_ARG,
              "tt2_synthesize_dev: null argument");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    TT2_HIP(hipMemcpyAsync(c->lens.p, lengths_d, sizeof(int) * B, hipMemcpyDeviceToDevice, s));
    const float* ref_d[2] = {ref_emt_d, ref_spk_d};
    const int trs[2] = {T_ref_emt, T_ref_spk};
    TT2_HIP(hipEventRecord(c->ev[0], s));
    encode_dev(c, ids_d, c->lens.as<int>(), lengths_host, B, T_in, ref_d, trs, s);
    TT2_HIP(hipEventRecord(c->ev[1], s));
    decode_dev(c, max_iters, prenet_masks_d, seed, nullptr, 0, c->frames.as<float>(),
               stop_d ? stop_d : c->stop.as<float>(), nullptr, s);
    TT2_HIP(hipEventRecord(c->ev[2], s));
    postnet_dev(c, c->frames.as<float>(), (long)max_iters * c->R * c->nm, B, c->n_steps * c->R, c->dec.as<float>(),
                mel_d, s);
    TT2_HIP(hipEventRecord(c->ev[3], s));
    c->timed = true;
    *n_steps_host = c->n_steps;
  });
}

tt2_status tt2_last_timings(tt2_ctx* c, float* ms3) {
  return guard([&] {
    TT2_CHECK(c && ms3, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->timed, TT2_ERR_STATE, "no timed tt2_synthesize_dev call yet");
    TT2_HIP(hipEventSynchronize(c->ev[3]));
    for (int i = 0; i < 3; ++i) TT2_HIP(hipEventElapsedTime(&ms3[i], c->ev[i], c->ev[i + 1]));
  });
}

#define TT2_NPROF 10

tt2_status tt2_profile_decoder_kernels(tt2_ctx* c, int iters, float* avg_us) {
  return guard([&] {
    TT2_CHECK(c && avg_us && iters >= 1, TT2_ERR_INVALID_ARG, "bad argument");
    TT2_CHECK(c->have_args, TT2_ERR_STATE, "tt2_profile_decoder_kernels needs a prior decode");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    DecArgs a = c->last_args;
    if (!g_stamps_dev) TT2_HIP(hipMalloc(&g_stamps_dev, 64 * sizeof(long long)));
    TT2_HIP(hipMemsetAsync(g_stamps_dev, 0, 64 * sizeof(long long), s));
    a.stamps = g_stamps_dev;
    a.frames = c->frames.as<float>();
    a.stop = c->stop.as<float>();
    a.align = nullptr;
    TT2_HIP(hipMemsetAsync(c->ctl.p, 0, sizeof(DecCtl), s));  // done = 0, tbase = 0
    hipEvent_t e0, e1;
    TT2_HIP(hipEventCreate(&e0));
    TT2_HIP(hipEventCreate(&e1));
    DecArgs a0 = a;
    a0.B = 0;  // energy launch with only its side-job blocks
    SideJob none = side_rec(c, 1, 0);
    none.ntile = 0;
    for (int k = 0; k < TT2_NPROF; ++k) {
      // `iters` back-to-back launches between one event pair: per-launch time = device
      // duration + the inter-kernel gap (comparable with rocprofv3 kernel-trace averages)
      TT2_HIP(hipMemsetAsync(c->ctl.p, 0, sizeof(DecCtl), s));
      TT2_HIP(hipEventRecord(e0, s));
      for (int i = 0; i < iters; ++i) {
        const int par = i & 1;
        switch (k) {
          case 0: launch_prenet(c, a, 0, 0, s); break;
          case 1: launch_lstm(lstm_args(c, a, par, 0), c->H, s); break;  // layers 1/2 alternating
          case 2: launch_query(c, a, none, s); break;
          case 3: launch_energy(c, a, side_rec(c, 1, 0), s); break;
          case 4: launch_softmax(c, a, 0, 0, side_rec(c, 0, 0), s); break;
          case 5: launch_proj(c, a, 0, none, s); break;
          case 6: launch_lstm(lstm_args(c, a, 1, 0), c->H, s); break;
          case 7: launch_energy(c, a0, side_rec(c, 1, 0), s); break;   // side job alone
          case 8: launch_energy(c, a, none, s); break;                 // energy alone
          case 9: launch_softmax(c, a, 0, 0, none, s); break;          // softmax alone
        }
      }
      TT2_HIP(hipEventRecord(e1, s));
      TT2_HIP(hipEventSynchronize(e1));
      float ms = 0.f;
      TT2_HIP(hipEventElapsedTime(&ms, e0, e1));
      avg_us[k] = 1000.f * ms / iters;
    }
    TT2_HIP(hipEventDestroy(e0));
    TT2_HIP(hipEventDestroy(e1));
    TT2_HIP(hipMemcpy(c->stamps_host, g_stamps_dev, 64 * sizeof(long long), hipMemcpyDeviceToHost));
    c->decoded = false;
  });
}

tt2_status tt2_hbm_copy_gbps(int hip_device, long long bytes, int iters, double* gbps) {
  return guard([&] {
    TT2_CHECK(gbps && bytes >= (1LL << 20) && iters >= 1, TT2_ERR_INVALID_ARG,
              "tt2_hbm_copy_gbps: bytes >= 1 MiB, iters >= 1, gbps non-null");
    TT2_HIP(hipSetDevice(hip_device));
    hipDeviceProp_t prop;
    TT2_HIP(hipGetDeviceProperties(&prop, hip_device));
    const long n4 = (long)(bytes / 16);
    DevBuf a, b;
    a.alloc((size_t)n4 * 16);
    b.alloc((size_t)n4 * 16);
    TT2_HIP(hipMemset(a.p, 0, (size_t)n4 * 16));
    hipStream_t s;
    TT2_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    TT2_HIP(hipEventCreate(&e0));
    TT2_HIP(hipEventCreate(&e1));
    // a few copy shapes (blocks in flight per CU x float4s in flight per thread x cache policy);
    // the best of all timed copies is the measured peak
    float best = 1e30f;
    for (int v = 0; v < 6; ++v) {
      const dim3 grid((unsigned)((v % 3 == 0 ? 4 : v % 3 == 1 ? 8 : 16) * prop.multiProcessorCount));
      for (int it = -1; it < iters; ++it) {  // it = -1: warm-up (page mapping, clocks)
        TT2_HIP(hipEventRecord(e0, s));
        if (v < 3) hipLaunchKernelGGL((k_hbm_copy<8, false>), grid, dim3(256), 0, s, a.as<f32x4>(), b.as<f32x4>(), n4);
        else hipLaunchKernelGGL((k_hbm_copy<8, true>), grid, dim3(256), 0, s, a.as<f32x4>(), b.as<f32x4>(), n4);
        TT2_HIP(hipGetLastError());
        TT2_HIP(hipEventRecord(e1, s));
        TT2_HIP(hipEventSynchronize(e1));
        float ms = 0.f;
        TT2_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 0) best = std::min(best, ms);
      }
    }
    TT2_HIP(hipEventDestroy(e0));
    TT2_HIP(hipEventDestroy(e1));
    TT2_HIP(hipStreamDestroy(s));
    *gbps = 2.0 * (double)n4 * 16.0 / ((double)best * 1e-3) / 1e9;
  });
}

tt2_status tt2_decoder_path(tt2_ctx* c, int* persistent, float* kernel_ms) {
  return guard([&] {
    TT2_CHECK(c && persistent && kernel_ms, TT2_ERR_INVALID_ARG, "null argument");
    *persistent = c->last_pd ? 1 : (pd_fits(c) ? 1 : 0);
    *kernel_ms = c->last_pd ? c->pd_kernel_ms : 0.f;
  });
}

tt2_status tt2_linear_outputs_dev(tt2_ctx* c, const float* mels_d, int B, int T, float* linear_d, void* stream) {
  return guard([&] {
    TT2_CHECK(c && mels_d && linear_d, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_finalize_weights not called");
    TT2_CHECK(B >= 1 && T >= 1, TT2_ERR_INVALID_ARG, "B and T must be >= 1");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    cbhg_linear(c->cbhg, mels_d, B, T, linear_d, c->kpart.as<float>(), (long)(c->kpart.bytes / sizeof(float)), s);
  });
}

tt2_status tt2_linear_outputs(tt2_ctx* c, const float* mels, int B, int T, float* linear_out) {
  return guard([&] {
    TT2_CHECK(c && mels && linear_out, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->finalized, TT2_ERR_NOT_LOADED, "tt2_finalize_weights not called");
    TT2_CHECK(B >= 1 && T >= 1, TT2_ERR_INVALID_ARG, "B and T must be >= 1");
    TT2_HIP(hipSetDevice(c->dev));
    hipStream_t s = c->stream;
    DevBuf in, out;
    in.alloc(sizeof(float) * (size_t)B * T * c->nm);
    out.alloc(sizeof(float) * (size_t)B * T * c->cfg.num_freq);
    TT2_HIP(hipMemcpyAsync(in.p, mels, in.bytes, hipMemcpyHostToDevice, s));
    cbhg_linear(c->cbhg, in.as<float>(), B, T, out.as<float>(), c->kpart.as<float>(),
                (long)(c->kpart.bytes / sizeof(float)), s);
    TT2_HIP(hipMemcpyAsync(linear_out, out.p, out.bytes, hipMemcpyDeviceToHost, s));
    TT2_HIP(hipStreamSynchronize(s));
  });
}

tt2_status tt2_set_emt_labels(tt2_ctx* c, const int32_t* labels, int B) {
  return guard([&] {
    TT2_CHECK(c && labels, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->emt.on(), TT2_ERR_STATE, "tt2_set_emt_labels: the context is not the Tacotron_emt_attn variant");
    TT2_CHECK(B >= 1 && B <= c->cfg.max_batch, TT2_ERR_SHAPE_MISMATCH, "batch exceeds capacity");
    for (int b = 0; b < B; ++b) c->emt_labels[b] = labels[b];
  });
}

tt2_status tt2_emt_alignments(tt2_ctx* c, float* out, int32_t* heads, int32_t* T_v) {
  return guard([&] {
    TT2_CHECK(c && heads && T_v, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(c->emt.on(), TT2_ERR_STATE, "tt2_emt_alignments: the context is not the Tacotron_emt_attn variant");
    TT2_CHECK(c->encoded, TT2_ERR_STATE, "tt2_emt_alignments called before tt2_encode");
    *heads = c->emt.heads;
    *T_v = c->emt.Tv;
    if (!out) return;
    TT2_CHECK(c->decoded, TT2_ERR_STATE, "tt2_emt_alignments called before tt2_decode");
    TT2_HIP(hipStreamSynchronize(c->stream));
    const size_t n = (size_t)std::min(c->n_steps, c->emt.max_iters) * c->B * c->emt.heads * c->emt.Tv;
    TT2_HIP(hipMemcpy(out, c->emt.hist.p, sizeof(float) * n, hipMemcpyDeviceToHost));
  });
}

tt2_status tt2_debug_pd_stamps(tt2_ctx* c, long long* out8192) {
  return guard([&] {
    TT2_CHECK(c && out8192, TT2_ERR_INVALID_ARG, "null argument");
    TT2_CHECK(g_pd_stamps_dev, TT2_ERR_STATE, "no persistent decode ran with TT2_STAMP_STEP set");
    TT2_HIP(hipDeviceSynchronize());
    TT2_HIP(hipMemcpy(out8192, g_pd_stamps_dev, PD_NB * 32 * sizeof(long long), hipMemcpyDeviceToHost));
  });
}

tt2_status tt2_debug_stamps(tt2_ctx* c, long long* out64) {
  return guard([&] {
    TT2_CHECK(c && out64, TT2_ERR_INVALID_ARG, "null argument");
    if (g_stamps_dev) {
      TT2_HIP(hipDeviceSynchronize());
      TT2_HIP(hipMemcpy(c->stamps_host, g_stamps_dev, 64 * sizeof(long long), hipMemcpyDeviceToHost));
    }
    for (int i = 0; i < 64; ++i) out64[i] = c->stamps_host[i];
  });
}

tt2_status tt2_output_lengths_dev(const float* stop_d, int B, int n_steps, int ld, int32_t* lengths_d, void* stream) {
  return guard([&] {
    TT2_CHECK(stop_d && lengths_d, TT2_ERR_INVALID_ARG, "tt2_output_lengths_dev: null argument");
    TT2_CHECK(B >= 1 && n_steps >= 0 && ld >= n_steps, TT2_ERR_SHAPE_MISMATCH, "tt2_output_lengths_dev: bad sizes");
    hipLaunchKernelGGL(k_output_lengths, dim3(B), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), stop_d, n_steps,
                       (long)ld, lengths_d);
    TT2_HIP(hipGetLastError());
  });
}

}  // extern "C"
