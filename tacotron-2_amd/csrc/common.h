// Shared device/host helpers for libtt2 (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/tt2.h"

namespace tt2 {

// ------------------------------------------------------------------------------------------
// Errors: HIP failures become exceptions inside the library and a status at the ABI.
// ------------------------------------------------------------------------------------------
struct Error : std::runtime_error {
  int status;
  Error(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

void set_last_error(const std::string& msg);

#define TT2_HIP(call)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess)                                                                  \
      throw ::tt2::Error(e_ == hipErrorOutOfMemory ? TT2_ERR_OOM : TT2_ERR_HIP,            \
                         std::string(#call) + ": " + hipGetErrorString(e_));               \
  } while (0)

#define TT2_CHECK(cond, status, msg)                                                       \
  do {                                                                                     \
    if (!(cond)) throw ::tt2::Error(status, msg);                                          \
  } while (0)

std::string redzone_check_all(const char* phase);  // TT2_REDZONE: every live buffer, unnamed

// Redzones (TT2_REDZONE=1, debug only): every DevBuf gets kRedzone extra bytes past its end filled
// with kRedByte; redzone_check() (called by the training entry points between phases) reports the
// first buffer whose redzone a kernel wrote -- the buffer that overflowed, whatever the address
// layout of the process puts behind it.
inline bool redzone_on() {
  static const bool on = [] {
    const char* e = std::getenv("TT2_REDZONE");
    return e && e[0] && e[0] != '0';
  }();
  return on;
}
template <class F>
tt2_status guard(F&& f) {
  try {
    f();
    if (redzone_on()) {  // debug: every ABI call leaves every live buffer's redzone intact
      const std::string r = redzone_check_all("ABI call");
      if (!r.empty()) throw Error(TT2_ERR_HIP, "redzone violation: " + r);
    }
    return TT2_OK;
  } catch (const Error& e) {
    set_last_error(e.what());
    return e.status;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return TT2_ERR_INVALID_ARG;
  }
}

// Debug fill of fresh allocations (TT2_POISON_ALLOC=1): every DevBuf starts as 0xFF bytes (fp32
// NaN, int -1, u8 255), so a kernel that reads a buffer before the call writes it shows up as a
// NaN / wrong value deterministically instead of depending on what an earlier allocation left.
// TT2_POISON_ALLOC=<byte> picks another fill (e.g. 66 = 0x42424242 = 48.6f, finite, so a stale read
// that a max / compare would swallow as NaN still changes the result).
inline int poison_alloc() {
  static const int fill = [] {
    const char* e = std::getenv("TT2_POISON_ALLOC");
    if (!e || !e[0] || (e[0] == '0' && !e[1])) return -1;
    const long v = std::strtol(e, nullptr, 0);
    return v == 1 ? 0xFF : (int)(v & 0xFF);
  }();
  return fill;
}

constexpr size_t kRedzone = 1 << 16;
constexpr unsigned char kRedByte = 0xA5;
struct DevBuf;
// "" = every registered redzone intact (defined in tacotron.hip); namer (may be null) names a buffer
std::string redzone_check(const char* phase, std::string (*namer)(const void* owner, const DevBuf* b),
                          const void* owner);
void redzone_register(DevBuf* b, bool add);

// Device buffer owned by a context.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { free(); }
  void alloc(size_t n) {
    if (n == bytes && p) return;
    free();
    if (n) {
      const bool rz = redzone_on();
      TT2_HIP(hipMalloc(&p, n + (rz ? kRedzone : 0)));
      if (poison_alloc() >= 0) TT2_HIP(hipMemset(p, poison_alloc(), n));
      if (rz) TT2_HIP(hipMemset(static_cast<char*>(p) + n, kRedByte, kRedzone));
      if (rz || poison_alloc() >= 0) TT2_HIP(hipDeviceSynchronize());
      bytes = n;
      if (rz) redzone_register(this, true);
    }
  }
  void free() {
    if (p) {
      if (redzone_on()) redzone_register(this, false);
      (void)hipFree(p);
    }
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Host-side store of loaded weights, keyed by TF variable name.
struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
};
using WeightMap = std::map<std::string, HostTensor>;

void put_tensor(WeightMap& wm, const char* name, const float* host, const int64_t* shape, int ndim);
const HostTensor& need(const WeightMap& wm, const std::string& name, std::vector<int64_t> shape);

// ------------------------------------------------------------------------------------------
// MFMA f32 fragment layouts (v_mfma_f32_16x16x4_f32).
//
// Lane l of a 64-lane wave supplies A[i=l&15][k=l>>4] and B[k=l>>4][j=l&15]; the 4 accumulator
// registers hold D[row=(l>>4)*4+r][col=l&15].
//
// "AF" activation layout of a 32-row block with K columns (K % 16 == 0): lane l of the wave that
// processes k-group sg (16 k's) and row-half h loads one float4 holding A[h*16+(l&15)]
// [16*sg + 4*j + (l>>4)] for j = 0..3 -> one 1 KiB coalesced load per (sg, h).
// "WF" weight layout of a 16-column tile: lane l loads float4 W[16*sg + 4*j + (l>>4)][l&15].
// ------------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline int af_idx(int m, int k) {
  const int s = k >> 2, kk = k & 3, h = m >> 4, i = m & 15;
  return ((((s >> 2) * 2 + h) * 64 + (kk * 16 + i)) << 2) + (s & 3);
}
__host__ __device__ inline int wf_idx(int k, int j) {  // within one 16-column tile
  const int s = k >> 2, kk = k & 3;
  return ((((s >> 2) * 64) + (kk * 16 + j)) << 2) + (s & 3);
}

// One k-group (16 k) of an AF x WF product as split fp16x3 MFMA: the AF/WF float4 of lane l holds
// k = 16sg + 4e + (l>>4) for both operands, so the same (l>>4, e) -> k map turns each hi/lo pair
// of float4s into valid v_mfma_f32_16x16x16_f16 operands; A·B = Ah·Bh + Ah·Bl + Al·Bh (fp32
// accumulation, fp16 products exact) -- 3 instead of 8 fp32 MFMAs' worth of issue per row half.
//
// Exact power-of-two pre-scale of the B operand (as gemm.hip's split16 path): the resident weights
// are stored pre-multiplied by KG_SB = 2^10 (the persistent decoder's weight copies at finalize,
// the BiLSTM's register fragments in its prologue), so the lo halves of weights down to ~1e-4
// (trained checkpoints: 1e-3..1e-1) stay fp16 normals instead of losing bits as subnormals; every
// accumulator fed by kg_mfma_x3 carries 2^10 and is multiplied by KG_UNSCALE where it is consumed.
// Valid for |B| < 64 (KG_BMAX, checked on the host at finalize: larger weights route to the
// fp32-MFMA launch path).  The A operand (activations: tanh/sigmoid-bounded h, context, prenet
// outputs) is split unscaled: its split error is <= 2^-25 absolute even where lo is subnormal,
// i.e. below fp32's own rounding of |a| >= 0.5 and at fp32-dot-product noise level below that
// (|a|·sqrt(K)·2^-25 against |a|·sqrt(K)·2^-24 rounding of the fp32 sum); pre-scaling it measured
// +1.1 us per decoder step (A/B, round 2) for no parity gain.
constexpr float KG_SB = 1024.f, KG_UNSCALE = 1.f / 1024.f, KG_BMAX = 63.9f;
typedef _Float16 kg_f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void kg_split(const f32x4& v, kg_f16x4& h, kg_f16x4& l) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 x = (_Float16)v[e];
    h[e] = x;
    l[e] = (_Float16)(v[e] - (float)x);
  }
}
// bw is the pre-scaled (x KG_SB) weight fragment; c0/c1 accumulate A·B·2^10.
__device__ __forceinline__ void kg_mfma_x3(const f32x4& a0, const f32x4& a1, const f32x4& bw, f32x4& c0,
                                           f32x4& c1) {
  kg_f16x4 a0h, a0l, a1h, a1l, bh, bl;
  kg_split(a0, a0h, a0l);
  kg_split(a1, a1h, a1l);
  kg_split(bw, bh, bl);
  c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a0l, bh, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a1l, bh, c1, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a0h, bl, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a1h, bl, c1, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a0h, bh, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a1h, bh, c1, 0, 0, 0);
}

// acc[h] += A(rows h*16..h*16+15, k in [16*sg0, 16*sg1)) * Wtile(k, 0..15)
__device__ __forceinline__ void skinny_mfma(const float* __restrict__ X, const float* __restrict__ Wt,
                                            int sg0, int sg1, f32x4& acc0, f32x4& acc1, int lane) {
  const f32x4* Xv = reinterpret_cast<const f32x4*>(X);
  const f32x4* Wv = reinterpret_cast<const f32x4*>(Wt);
#pragma unroll 4
  for (int sg = sg0; sg < sg1; ++sg) {
    const f32x4 a0 = Xv[(sg * 2 + 0) * 64 + lane];
    const f32x4 a1 = Xv[(sg * 2 + 1) * 64 + lane];
    const f32x4 b = Wv[sg * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], b[j], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], b[j], acc1, 0, 0, 0);
    }
  }
}

// Same product with every load of the wave's NPW k-groups issued before the first MFMA, so the
// whole K-slice (3 KiB per k-group per wave) is in flight at once; hipcc emits counted vmcnt waits.
template <int NPW>
__device__ __forceinline__ void skinny_mfma_all(const float* __restrict__ X, const float* __restrict__ Wt,
                                                int sg0, f32x4& acc0, f32x4& acc1, int lane) {
  const f32x4* Xv = reinterpret_cast<const f32x4*>(X);
  const f32x4* Wv = reinterpret_cast<const f32x4*>(Wt);
  f32x4 a0[NPW], a1[NPW], b[NPW];
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    b[j] = Wv[(sg0 + j) * 64 + lane];
    a0[j] = Xv[((sg0 + j) * 2 + 0) * 64 + lane];
    a1[j] = Xv[((sg0 + j) * 2 + 1) * 64 + lane];
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every load ahead of the first MFMA
#pragma unroll
  for (int j = 0; j < NPW; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j][e], b[j][e], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j][e], b[j][e], acc1, 0, 0, 0);
    }
}

// acc += X (LDS/global AF, k-groups [0, nsg)) * pre-loaded weight fragments w[0..nsg)
template <int MAXK>
__device__ __forceinline__ void skinny_mfma_w(const float* __restrict__ X, const f32x4* w, int nsg,
                                              f32x4& acc0, f32x4& acc1, int lane) {
  const f32x4* Xv = reinterpret_cast<const f32x4*>(X);
#pragma unroll
  for (int j = 0; j < MAXK; ++j) {
    if (j >= nsg) break;
    const f32x4 a0 = Xv[(j * 2 + 0) * 64 + lane];
    const f32x4 a1 = Xv[(j * 2 + 1) * 64 + lane];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[e], w[j][e], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[e], w[j][e], acc1, 0, 0, 0);
    }
  }
}

// Reduce the (acc0, acc1) of NW waves (each covering a K slice) through LDS into
// out[m*16 + n] (32 x 16), summing waves in index order (deterministic).
template <int NW>
__device__ __forceinline__ void reduce_waves_32x16(const f32x4& acc0, const f32x4& acc1, float* lds,
                                                   float* out, int wave, int lane, int tid) {
  // lds: NW * 512 floats
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int n = lane & 15, m = (lane >> 4) * 4 + r;
    lds[wave * 512 + m * 16 + n] = acc0[r];
    lds[wave * 512 + (m + 16) * 16 + n] = acc1[r];
  }
  __syncthreads();
  for (int e = tid; e < 512; e += NW * 64) {
    float s = lds[e];
#pragma unroll
    for (int w = 1; w < NW; ++w) s += lds[w * 512 + e];
    out[e] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
// tanh from one v_exp_f32 + one division: |abs err| < 2e-7 over the whole range (the location-
// sensitive energy evaluates 32x128 of these per 32 encoder steps; libm tanhf costs ~10x more)
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __expf(2.0f * x);
  return 1.0f - 2.0f / (e + 1.0f);
}
// Accurate variants used where parity matters (expf is correctly-rounded-ish ocml).
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

#define TT2_HD __host__ __device__
#include "rng.h"

// Gaussian head: the N(0,1) draw of Normal.sample (gaussian.py:50), Box-Muller on channels 14, 15.
__device__ inline float wn_gauss(uint64_t seed, long t, int Bg, int b) {
  const float u1 = wn_uniform(seed, t, Bg, b, 14), u2 = wn_uniform(seed, t, Bg, b, 15);
  return sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// Persistent kernels (their work-groups spin on each other's hand-offs) launch cooperatively, which
// makes the runtime refuse a grid that cannot be co-resident.  TT2_COOP=0 launches the same grid
// with hipLaunchKernel (after the same occupancy checks): a diagnostic switch for profiler runs.
inline hipError_t launch_persistent(const void* f, dim3 grid, dim3 block, void** args, size_t shm, hipStream_t s) {
  static const bool coop = !(getenv("TT2_COOP") && atoi(getenv("TT2_COOP")) == 0);
  return coop ? hipLaunchCooperativeKernel(f, grid, block, args, (unsigned)shm, s)
              : hipLaunchKernel(f, grid, block, args, shm, s);
}

// ------------------------------------------------------------------------------------------
// DPP cross-lane reductions inside one 16-lane row (VALU only, no LDS round trip).  Every step
// adds a value and its mirror partner, so all 16 lanes end with bitwise-identical sums.
// ------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_XOR1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141; // row_half_mirror
constexpr int DPP_MIRROR = 0x140;      // row_mirror
__device__ __forceinline__ float sum16(float v) {
  v += dpp_f<DPP_XOR1>(v);
  v += dpp_f<DPP_XOR2>(v);
  v += dpp_f<DPP_HALF_MIRROR>(v);
  v += dpp_f<DPP_MIRROR>(v);
  return v;
}
__device__ __forceinline__ void sum16x4(f32x4& a) {
#define TT2_STEP(C)                                                                                  \
  {                                                                                                  \
    const float t0 = dpp_f<C>(a[0]), t1 = dpp_f<C>(a[1]), t2 = dpp_f<C>(a[2]), t3 = dpp_f<C>(a[3]); \
    a[0] += t0; a[1] += t1; a[2] += t2; a[3] += t3;                                                  \
  }
  TT2_STEP(DPP_XOR1) TT2_STEP(DPP_XOR2) TT2_STEP(DPP_HALF_MIRROR) TT2_STEP(DPP_MIRROR)
#undef TT2_STEP
}
// wave-uniform max / sum of 64 lanes from DPP row operations + the two row broadcasts (no LDS
// round trip as __shfl_xor's ds_bpermute): the masked-off rows keep their own value
template <int CTRL, int RMASK>
__device__ __forceinline__ float dpp_keep(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, RMASK, 0xF, false));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f<DPP_XOR1>(v));
  v = fmaxf(v, dpp_f<DPP_XOR2>(v));
  v = fmaxf(v, dpp_f<DPP_HALF_MIRROR>(v));
  v = fmaxf(v, dpp_f<DPP_MIRROR>(v));
  v = fmaxf(v, dpp_keep<0x142, 0xA>(v));  // row_bcast:15
  v = fmaxf(v, dpp_keep<0x143, 0xC>(v));  // row_bcast:31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = sum16(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// after sum16: lane 31 of each 32-lane half holds that half's sum (rows 0+1, rows 2+3)
__device__ __forceinline__ float sum32_to_lane31(float v) {
  v = sum16(v);
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));  // row_bcast:15
}
// full 64-lane sum, valid in lane 63
__device__ __forceinline__ float sum64_to_lane63(float v) {
  v = sum32_to_lane31(v);
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));  // row_bcast:31
}
// Gate non-linearities from v_exp_f32 + v_rcp_f32 (no branches, no IEEE division): abs error
// < 3e-7 for tanh, relative error < 4e-7 for the sigmoid over the whole range.
__device__ __forceinline__ float sigm_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_rcp(float x) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * x) + 1.0f);
}
// argmax over a 16-lane row, ties -> lowest index (tf.argmax); result in every lane of the row
__device__ __forceinline__ void argmax16(float& v, int& i) {
#define TT2_STEP(C)                                                    \
  {                                                                    \
    const float ov = dpp_f<C>(v);                                      \
    const int oi = dpp_i<C>(i);                                        \
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }             \
  }
  TT2_STEP(DPP_XOR1) TT2_STEP(DPP_XOR2) TT2_STEP(DPP_HALF_MIRROR) TT2_STEP(DPP_MIRROR)
#undef TT2_STEP
}

}  // namespace tt2
