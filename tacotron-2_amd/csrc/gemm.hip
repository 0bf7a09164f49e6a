// fp32 GEMM on the CDNA4 matrix cores: exact fp32 (v_mfma_f32_32x32x2_f32) or split fp16x3
// (v_mfma_f32_32x32x16_f16 on hi/lo halves, GemmArgs::split16).
//
// C[M,N] = epilogue(A[M,K] · B[K,N]).  A is read through an implicit-im2col loader (dense rows,
// 'same' conv1d, NHWC conv2d) so the encoder/postnet/refnet convolutions never materialise their
// column matrices in HBM.  Block tile (64·WMB)×(64·WNB)×16, 4 waves in a 2×2 grid, each wave owns
// WMB×WNB 32×32 accumulators; LDS double-buffered, next tile prefetched into registers while the
// current one is multiplied.
#include "gemm.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <cstdio>

namespace tt2 {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <bool VA>
__device__ __forceinline__ void load_a4(const GemmArgs& g, int m, int k, float* v) {
  v[0] = v[1] = v[2] = v[3] = 0.f;
  if (m >= g.M || k >= g.K) return;
  if (g.a_mode == A_DENSE) {
    const float* p = g.A + (long)m * g.lda + k;
    if (VA && k + 3 < g.K) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(p);
      v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
    } else {
      for (int i = 0; i < 4; ++i)
        if (k + i < g.K) v[i] = p[i];
    }
    return;
  }
  if (g.a_mode == A_CONV1D) {
    const int b = m / g.T, t = m - b * g.T;
    if (VA && k + 3 < g.K) {  // C % 4 == 0: the 4 k's share one tap
      const int tap = k / g.C, c = k - tap * g.C;
      const int tt = t + tap - g.pad;
      if (tt >= 0 && tt < g.T) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(g.A + b * g.xs_b + (long)tt * g.xs_t + c);
        v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
      }
    } else {
      for (int i = 0; i < 4; ++i) {
        const int kk = k + i;
        if (kk >= g.K) break;
        const int tap = kk / g.C, c = kk - tap * g.C;
        const int tt = t + tap - g.pad;
        if (tt >= 0 && tt < g.T) v[i] = g.A[b * g.xs_b + (long)tt * g.xs_t + c];
      }
    }
    return;
  }
  // A_CONV2D (NHWC)
  const int hw = g.Ho * g.Wo;
  const int n = m / hw, r = m - n * hw, ho = r / g.Wo, wo = r - ho * g.Wo;
  if (VA && k + 3 < g.K) {
    const int ij = k / g.C, c = k - ij * g.C, i = ij / g.kw2, j = ij - i * g.kw2;
    const int h = ho * g.sh + i - g.pt, w = wo * g.sw + j - g.pl;
    if (h >= 0 && h < g.H && w >= 0 && w < g.Wd) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(g.A + (((long)n * g.H + h) * g.Wd + w) * g.C + c);
      v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
    }
  } else {
    for (int e = 0; e < 4; ++e) {
      const int kk = k + e;
      if (kk >= g.K) break;
      const int ij = kk / g.C, c = kk - ij * g.C, i = ij / g.kw2, j = ij - i * g.kw2;
      const int h = ho * g.sh + i - g.pt, w = wo * g.sw + j - g.pl;
      if (h >= 0 && h < g.H && w >= 0 && w < g.Wd) v[e] = g.A[(((long)n * g.H + h) * g.Wd + w) * g.C + c];
    }
  }
}

template <bool VB>
__device__ __forceinline__ void load_b4(const GemmArgs& g, int k, int n, float* v) {
  v[0] = v[1] = v[2] = v[3] = 0.f;
  if (k >= g.K || n >= g.N) return;
  const float* p = g.Bw + (long)k * g.ldb + n;
  if (VB && n + 3 < g.N) {
    const f32x4 q = *reinterpret_cast<const f32x4*>(p);
    v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
  } else {
    for (int i = 0; i < 4; ++i)
      if (n + i < g.N) v[i] = p[i];
  }
}

// Static weights for split16 == 1: B [K][N] fp32 -> pre-scaled (x2^10), split fp16 planes
// transposed to [N][ldbt] (k contiguous): one 16-byte load per 8 k in the GEMM, no per-call split.
__global__ void k_split_bt(const float* __restrict__ B, int K, int N, long ldb, long ldbt, _Float16* __restrict__ hi,
                           _Float16* __restrict__ lo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * ldbt) return;
  const int n = (int)(i / ldbt), k = (int)(i % ldbt);
  const float x = k < K ? B[(long)k * ldb + n] * 1024.f : 0.f;
  const _Float16 h = (_Float16)x;
  hi[i] = h;
  lo[i] = (_Float16)(x - (float)h);
}

// Fused epilogue of one 32x32 accumulator tile (C/D layout: col = lane&31,
// row = (r&3) + 8*(r>>2) + 4*(lane>>5), identical for the f32 and f16 MFMA shapes on gfx950).
__device__ __forceinline__ void epilogue_tile(const GemmArgs& g, const f32x16& acc, int row0, int col0, int lane) {
  const int col = col0 + (lane & 31);
  if (col >= g.N) return;
  const float bias = g.bias ? g.bias[col] : 0.f;
  const float sc = g.bn_scale ? g.bn_scale[col] : 1.f;
  const float sh = g.bn_shift ? g.bn_shift[col] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row >= g.M) continue;
    float y = acc[r] + bias;
    if (g.act == ACT_RELU) y = fmaxf(y, 0.f);
    else if (g.act == ACT_TANH) y = tanhf(y);
    if (g.bn_scale) y = y * sc + sh;
    if (g.act == ACT_BN_RELU) y = fmaxf(y, 0.f);  // BN then ReLU (conv2d(), modules.py:507-510)
    if (g.residual) y = g.residual[(long)row * g.ldr + col] + y;
    if (g.clip) y = fminf(fmaxf(y, g.clip_lo), g.clip_hi);
    g.Cout[(long)row * g.ldc + col] = y;
  }
}

template <int WMB, int WNB, bool VA, bool VB>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  constexpr int BM = 64 * WMB, BN = 64 * WNB, BK = 16;
  constexpr int EA = BM * BK / 256, TPR_A = BK / EA;
  constexpr int EB = BN * BK / 256, TPR_B = BN / EB;
  __shared__ float As[2][BK][BM + 4];
  __shared__ float Bs[2][BK][BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int am = tid / TPR_A, ak = (tid % TPR_A) * EA;
  const int bk = tid / TPR_B, bn = (tid % TPR_B) * EB;
  float ra[EA], rb[EB];
  f32x16 acc[WMB][WNB];
#pragma unroll
  for (int i = 0; i < WMB; ++i)
#pragma unroll
    for (int j = 0; j < WNB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto gload = [&](int k0) {
#pragma unroll
    for (int e = 0; e < EA; e += 4) load_a4<VA>(g, m0 + am, k0 + ak + e, &ra[e]);
#pragma unroll
    for (int e = 0; e < EB; e += 4) load_b4<VB>(g, k0 + bk, n0 + bn + e, &rb[e]);
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int e = 0; e < EA; ++e) As[buf][ak + e][am] = ra[e];
#pragma unroll
    for (int e = 0; e < EB; ++e) Bs[buf][bk][bn + e] = rb[e];
  };

  // split-K: this block covers k tiles [kt0, kt1) (g.K clipped so the loaders zero-fill past it)
  const int nkt = (g.K + BK - 1) / BK;
  const int per = (nkt + g.ksplit - 1) / g.ksplit;
  const int kt0 = blockIdx.z * per, kt1 = min(nkt, kt0 + per);
  if (g.ksplit > 1) g.K = min(g.K, kt1 * BK);
  const int nk = kt1 - kt0;
  if (nk > 0) {
  gload(kt0 * BK);
  sstore(0);
  __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt0 + kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[WMB], b[WNB];
#pragma unroll
      for (int i = 0; i < WMB; ++i) a[i] = As[cur][kk + (lane >> 5)][wm * 32 * WMB + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < WNB; ++j) b[j] = Bs[cur][kk + (lane >> 5)][wn * 32 * WNB + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < WMB; ++i)
#pragma unroll
        for (int j = 0; j < WNB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  if (g.ksplit > 1 || g.raw) {  // raw partial tile -> kpart[z][M][N]
    float* P = g.kpart + (long)blockIdx.z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < WMB; ++i)
#pragma unroll
      for (int j = 0; j < WNB; ++j) {
        const int col = n0 + wn * 32 * WNB + j * 32 + (lane & 31);
        if (col >= g.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 32 * WMB + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < g.M) P[(long)row * g.N + col] = acc[i][j][r];
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < WMB; ++i)
#pragma unroll
    for (int j = 0; j < WNB; ++j)
      epilogue_tile(g, acc[i][j], m0 + wm * 32 * WMB + i * 32, n0 + wn * 32 * WNB + j * 32, lane);
}

// split-K combine: C = epilogue(sum_z kpart[z]) (same epilogue as epilogue_tile)
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmArgs g) {
  // 4 consecutive outputs per thread: 16-byte partial loads when N % 4 == 0, eight independent
  // accumulator chains over the splits (8 loads in flight per round, not a dependent chain)
  const long MN = (long)g.M * g.N;
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i0 >= MN) return;
  float y[4] = {0.f, 0.f, 0.f, 0.f};
  if ((g.N & 3) == 0) {
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    f32x4 a[8] = {z4, z4, z4, z4, z4, z4, z4, z4};
    for (int z0 = 0; z0 < g.ksplit; z0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (z0 + u < g.ksplit) a[u] += *reinterpret_cast<const f32x4*>(g.kpart + (long)(z0 + u) * MN + i0);
    }
    const f32x4 t = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = t[e];
  } else {
    for (int e = 0; e < 4 && i0 + e < MN; ++e)
      for (int z = 0; z < g.ksplit; ++z) y[e] += g.kpart[(long)z * MN + i0 + e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long i = i0 + e;
    if (i >= MN) break;
    const int row = (int)(i / g.N), col = (int)(i % g.N);
    float v = y[e];
    if (g.bias) v += g.bias[col];
    if (g.act == ACT_RELU) v = fmaxf(v, 0.f);
    else if (g.act == ACT_TANH) v = tanhf(v);
    if (g.bn_scale) v = v * g.bn_scale[col] + g.bn_shift[col];
    if (g.act == ACT_BN_RELU) v = fmaxf(v, 0.f);
    if (g.residual) v = g.residual[(long)row * g.ldr + col] + v;
    if (g.clip) v = fminf(fmaxf(v, g.clip_lo), g.clip_hi);
    g.Cout[(long)row * g.ldc + col] = v;
  }
}


// ---- split fp16x3 GEMM (GemmArgs::split16) -------------------------------------------------
// Block 128x128x32, 4 waves in a 2x2 grid, each wave 2x2 tiles of 32x32 (v_mfma_f32_32x32x16_f16:
// lane l holds A[row l&31][k = 8(l>>5) + j] and B[k = 8(l>>5) + j][col l&31], j < 8).  Operands are
// split into fp16 hi/lo planes when staged into LDS ([row][k] for A, [col][k] for B, k contiguous:
// one ds_read_b128 per fragment), LDS double-buffered, next tile prefetched into registers.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int X3_BK = 32, X3_LD = X3_BK + 8;  // padded k stride (halfs)
// Operands are pre-scaled by powers of two before the split (A x2^4, B x2^10, result x2^-14,
// exact): an unscaled lo of a 1e-3 weight is an fp16 subnormal with ~1% precision, which cost up
// to 3e-5 relative error; scaled, the split is ~1e-7 relative for |A| < 4e3, |B| < 64.
constexpr float X3_SA = 16.f, X3_SB = 1024.f, X3_UNSCALE = 1.f / (16.f * 1024.f);

__device__ __forceinline__ void split8(const float* v, float scale, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = v[e] * scale;
    const _Float16 h = (_Float16)x;
    hi[e] = h;
    lo[e] = (_Float16)(x - (float)h);
  }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void to_bf16x8(const float* v, bf16x8& o) {
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];  // round to nearest even
}

// MODE 1: split fp16x3 (fp32-accurate); MODE 2: bf16 operands (one v_mfma_f32_32x32x16_bf16 per
// k-slab, fp32 accumulation -- the mixed-precision training GEMM).  Block (64·WMB) x 128 x 32,
// 4 waves in a 2x2 grid, each wave WMB x 2 tiles of 32x32; split-K over blockIdx.z as in
// gemm_kernel (raw partials to kpart, epilogue in gemm_splitk_reduce).
template <bool VA, int MODE, int WMB, bool BT = false>
__global__ __launch_bounds__(256) void gemm_x3_kernel(GemmArgs g) {
  constexpr int BM = 64 * WMB, BN = 128, BK = X3_BK;
  constexpr int EA = BM * BK / 256;            // A elements per thread (16 or 8)
  constexpr int TPR_A = BK / EA;               // threads per A row
  constexpr int NPL = MODE == 1 ? 2 : 1;       // hi/lo planes
  typedef typename std::conditional<MODE == 1, _Float16, __bf16>::type ET;
  typedef typename std::conditional<MODE == 1, f16x8, bf16x8>::type V8;
  __shared__ __attribute__((aligned(16))) ET As[NPL][2][BM][X3_LD];
  __shared__ __attribute__((aligned(16))) ET Bs[NPL][2][BN][X3_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int am = tid / TPR_A, ak = (tid % TPR_A) * EA;  // A: row am, k [ak, ak+EA)
  const int bn = tid & 127, bk = (tid >> 7) * 16;       // B: col bn, k [bk, bk+16) (coalesced over n)
  float ra[EA], rb[16];
  bf16x8 rbt[2];  // MODE 2 with Bt16: 16 pre-converted k values of column n
  f16x8 rbh[2], rbl[2];  // MODE 1 with Bt16/Bt16lo: 16 pre-split (hi, lo) k values of column n
  constexpr bool bt = MODE == 2 && BT;   // B from g.Bt16 (pre-transposed bf16)
  constexpr bool bt1 = MODE == 1 && BT;  // B from pre-scaled, pre-split fp16 planes
  f32x16 acc[WMB][2];
#pragma unroll
  for (int i = 0; i < WMB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto gload = [&](int k0) {
#pragma unroll
    for (int e = 0; e < EA; e += 4) load_a4<VA>(g, m0 + am, k0 + ak + e, &ra[e]);
    const int n = n0 + bn;
    if constexpr (bt1) {
      const long off = (long)n * g.ldbt + k0 + bk;
      const _Float16* sh = reinterpret_cast<const _Float16*>(g.Bt16) + off;
      const _Float16* sl = reinterpret_cast<const _Float16*>(g.Bt16lo) + off;
      const int k = k0 + bk;
      if (n < g.N && k + 16 <= g.K) {
        rbh[0] = *reinterpret_cast<const f16x8*>(sh);
        rbh[1] = *reinterpret_cast<const f16x8*>(sh + 8);
        rbl[0] = *reinterpret_cast<const f16x8*>(sl);
        rbl[1] = *reinterpret_cast<const f16x8*>(sl + 8);
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const bool ok = n < g.N && k + e < g.K;
          const _Float16 vh = ok ? sh[e] : (_Float16)0.f, vl = ok ? sl[e] : (_Float16)0.f;
          if (e < 8) { rbh[0][e] = vh; rbl[0][e] = vl; } else { rbh[1][e - 8] = vh; rbl[1][e - 8] = vl; }
        }
      }
      return;
    }
    if constexpr (bt) {
      const __bf16* src = reinterpret_cast<const __bf16*>(g.Bt16) + (long)n * g.ldbt + k0 + bk;
      const int k = k0 + bk;
      if (n < g.N && k + 16 <= g.K) {
        rbt[0] = *reinterpret_cast<const bf16x8*>(src);
        rbt[1] = *reinterpret_cast<const bf16x8*>(src + 8);
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const __bf16 v = (n < g.N && k + e < g.K) ? src[e] : (__bf16)0.f;
          if (e < 8) rbt[0][e] = v; else rbt[1][e - 8] = v;
        }
      }
      return;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int k = k0 + bk + e;
      rb[e] = (n < g.N && k < g.K) ? g.Bw[(long)k * g.ldb + n] : 0.f;
    }
  };
  auto sstore = [&](int buf) {
    if constexpr (MODE == 1) {
      f16x8 h, l;
#pragma unroll
      for (int q = 0; q < EA / 8; ++q) {
        split8(&ra[8 * q], X3_SA, h, l);
        *reinterpret_cast<f16x8*>(&As[0][buf][am][ak + 8 * q]) = h;
        *reinterpret_cast<f16x8*>(&As[1][buf][am][ak + 8 * q]) = l;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if constexpr (bt1) {
          h = rbh[q];
          l = rbl[q];
        } else {
          split8(&rb[8 * q], X3_SB, h, l);
        }
        *reinterpret_cast<f16x8*>(&Bs[0][buf][bn][bk + 8 * q]) = h;
        *reinterpret_cast<f16x8*>(&Bs[1][buf][bn][bk + 8 * q]) = l;
      }
    } else {
      bf16x8 h;
#pragma unroll
      for (int q = 0; q < EA / 8; ++q) {
        to_bf16x8(&ra[8 * q], h);
        *reinterpret_cast<bf16x8*>(&As[0][buf][am][ak + 8 * q]) = h;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if constexpr (bt) {
          h = rbt[q];
        } else {
          to_bf16x8(&rb[8 * q], h);
        }
        *reinterpret_cast<bf16x8*>(&Bs[0][buf][bn][bk + 8 * q]) = h;
      }
    }
  };

  const int nkt = (g.K + BK - 1) / BK;
  const int per = (nkt + g.ksplit - 1) / g.ksplit;
  const int kt0 = blockIdx.z * per, kt1 = min(nkt, kt0 + per);
  if (g.ksplit > 1) g.K = min(g.K, kt1 * BK);
  const int nk = kt1 - kt0;
  if (nk > 0) {
    gload(kt0 * BK);
    sstore(0);
    __syncthreads();
  }
  const int r = lane & 31, h8 = (lane >> 5) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt0 + kt + 1) * BK);
#pragma unroll
    for (int s16 = 0; s16 < BK; s16 += 16) {
      V8 ah[WMB], bh[2];
#pragma unroll
      for (int i = 0; i < WMB; ++i) ah[i] = *reinterpret_cast<const V8*>(&As[0][cur][wm * 32 * WMB + i * 32 + r][s16 + h8]);
#pragma unroll
      for (int j = 0; j < 2; ++j) bh[j] = *reinterpret_cast<const V8*>(&Bs[0][cur][wn * 64 + j * 32 + r][s16 + h8]);
      if constexpr (MODE == 1) {
        V8 al[WMB], bl[2];
#pragma unroll
        for (int i = 0; i < WMB; ++i)
          al[i] = *reinterpret_cast<const V8*>(&As[NPL - 1][cur][wm * 32 * WMB + i * 32 + r][s16 + h8]);
#pragma unroll
        for (int j = 0; j < 2; ++j) bl[j] = *reinterpret_cast<const V8*>(&Bs[NPL - 1][cur][wn * 64 + j * 32 + r][s16 + h8]);
#pragma unroll
        for (int i = 0; i < WMB; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int i = 0; i < WMB; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int i = 0; i < WMB; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] *= X3_UNSCALE;
  }
  if (g.ksplit > 1 || g.raw) {  // raw partial tile -> kpart[z][M][N]
    float* P = g.kpart + (long)blockIdx.z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < WMB; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + (lane & 31);
        if (col >= g.N) continue;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = m0 + wm * 32 * WMB + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
          if (row < g.M) P[(long)row * g.N + col] = acc[i][j][q];
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < WMB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) epilogue_tile(g, acc[i][j], m0 + wm * 32 * WMB + i * 32, n0 + wn * 64 + j * 32, lane);
}

// ---- skinny bf16 product (training: M <= 64 rows per decoder step) ---------------------------
// C[M<=64][N] = A[M][K] (fp32, rounded to bf16 as staged) · B (pre-transposed bf16 Bt16[N][ldbt]).
// One work-group = 64 rows x 64 columns x one K slice (blockIdx.z), 4 waves of one 32x32
// v_mfma_f32_32x32x16_bf16 accumulator each.  The WHOLE K slice of both operands is staged into LDS
// in one burst (every thread issues all its loads before any LDS write) -- the round trip to HBM /
// MALL is paid once per work-group instead of once per 32-deep k tile, which is what bound the
// 64x128x32 double-buffered kernel (gemm_x3_kernel) at these shapes.  The host picks the K split so
// the grid stays near one work-group per CU and the slice fits LDS; partials [z][M][N] as in
// gemm_x3_kernel (combined by the caller or gemm_splitk_reduce), or the epilogue when unsplit.
constexpr int SK_BN = 64, SK_BM = 64, SK_GMAX = 19;  // groups of 8 per thread: 64 x 608 / 8 / 256
__host__ __device__ constexpr int sk_ld(int kslice) { return kslice + 8; }  // padded k stride (bf16)
size_t sk_lds_bytes(int kslice) { return (size_t)(SK_BM + SK_BN) * sk_ld(kslice) * 2; }

template <bool VA>
__global__ __launch_bounds__(256, 1) void gemm_sk_kernel(GemmArgs g, int kslice) {
  extern __shared__ __attribute__((aligned(16))) __bf16 sk_sm[];
  const int KP = sk_ld(kslice);
  __bf16* As = sk_sm;               // [64][KP]
  __bf16* Bs = sk_sm + SK_BM * KP;  // [64][KP]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * SK_BN, k0 = blockIdx.z * kslice;
  const int g8 = kslice >> 3;  // 8-element groups per row of the slice
  const int ng = 64 * g8;      // groups per operand tile (A and B alike: 64 rows / columns)
  // every load of both operands is issued before the first LDS write: one round trip to
  // HBM / MALL per work-group (one wave per SIMD, so the staging registers are affordable)
  f32x4 va[SK_GMAX][2];
  bf16x8 vb[SK_GMAX];
  const __bf16* Bt = reinterpret_cast<const __bf16*>(g.Bt16);
#pragma unroll
  for (int u = 0; u < SK_GMAX; ++u) {
    const int idx = tid + 256 * u;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    va[u][0] = z;
    va[u][1] = z;
    for (int e = 0; e < 8; ++e) vb[u][e] = (__bf16)0.f;
    if (idx < ng) {
      const int r = idx / g8, kk = (idx - r * g8) * 8, k = k0 + kk;
      if (r < g.M) {
        const float* p = g.A + (long)r * g.lda + k;
        if (VA && k + 8 <= g.K) {
          va[u][0] = *reinterpret_cast<const f32x4*>(p);
          va[u][1] = *reinterpret_cast<const f32x4*>(p + 4);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (k + e < g.K) va[u][e >> 2][e & 3] = p[e];
        }
      }
      const int n = n0 + r;  // B: column r of the tile
      if (n < g.N) {
        const __bf16* q = Bt + (long)n * g.ldbt + k;
        if (k + 8 <= g.K) {
          vb[u] = *reinterpret_cast<const bf16x8*>(q);
        } else {
          for (int e = 0; e < 8; ++e)
            if (k + e < g.K) vb[u][e] = q[e];
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < SK_GMAX; ++u) {
    const int idx = tid + 256 * u;
    if (idx < ng) {
      const int r = idx / g8, kk = (idx - r * g8) * 8;
      bf16x8 h;
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = (__bf16)va[u][e >> 2][e & 3];
      *reinterpret_cast<bf16x8*>(As + r * KP + kk) = h;
      *reinterpret_cast<bf16x8*>(Bs + r * KP + kk) = vb[u];
    }
  }
  __syncthreads();
  const int rw = (w & 1) * 32, cw = (w >> 1) * 32, r = lane & 31, h8 = (lane >> 5) * 8;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  const __bf16* pa = As + (rw + r) * KP + h8;
  const __bf16* pb = Bs + (cw + r) * KP + h8;
  for (int kk = 0; kk < kslice; kk += 16) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(pa + kk);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(pb + kk);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
  if (g.ksplit > 1 || g.raw) {
    float* P = g.kpart + (long)blockIdx.z * g.M * g.N;
    const int col = n0 + cw + (lane & 31);
    if (col < g.N) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = rw + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
        if (row < g.M) P[(long)row * g.N + col] = acc[q];
      }
    }
    return;
  }
  epilogue_tile(g, acc, rw, n0 + cw, lane);
}

// ---- register-direct skinny bf16 product (training: M <= 64 rows per decoder step) -------------
// C[M<=64][N] = A[M][K] (fp32, rounded to bf16 as staged) · B (pre-transposed bf16 Bt16[N][ldbt]).
// One work-group = 64 rows x 128 columns x one K slice (blockIdx.z) of <= 32·RD_KT; wave w owns
// columns [32w, 32w+32) as 4 x 2 v_mfma_f32_16x16x32_bf16 accumulators.  The B fragments are loaded
// straight from Bt16 into registers (a lane's 8 k of one column are 16 contiguous bytes in the
// pre-transposed layout: no LDS round trip, no barrier between the weight stream and the MFMAs),
// the whole slice at once; only A (64 rows, shared by the 4 waves, L2-resident) is staged in LDS.
constexpr int RD_BN = 128, RD_KT = 12;
constexpr int RD_AG = (64 * RD_KT * 32 / 8 + 255) / 256;  // 8-element A groups per thread (12)
__host__ __device__ constexpr int rd_ld(int kslice) { return kslice + 8; }  // padded k stride (bf16)
size_t rd_lds_bytes(int kslice) { return (size_t)64 * rd_ld(kslice) * 2; }

__device__ __forceinline__ void epilogue_one(const GemmArgs& g, int row, int col, float acc) {
  float y = acc + (g.bias ? g.bias[col] : 0.f);
  if (g.act == ACT_RELU) y = fmaxf(y, 0.f);
  else if (g.act == ACT_TANH) y = tanhf(y);
  if (g.bn_scale) y = y * g.bn_scale[col] + g.bn_shift[col];
  if (g.act == ACT_BN_RELU) y = fmaxf(y, 0.f);
  if (g.residual) y = g.residual[(long)row * g.ldr + col] + y;
  if (g.clip) y = fminf(fmaxf(y, g.clip_lo), g.clip_hi);
  g.Cout[(long)row * g.ldc + col] = y;
}

__global__ __launch_bounds__(256, 1) void gemm_rd_kernel(GemmArgs g, int kslice) {
  extern __shared__ __attribute__((aligned(16))) __bf16 rd_sm[];
  const int LD = rd_ld(kslice);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * RD_BN, k0 = blockIdx.z * kslice;
  const int kend = min(g.K, k0 + kslice);
  const int nks = (kend - k0 + 31) >> 5;  // 32-deep steps of this slice (<= RD_KT, host-checked)
  const int g8 = kslice >> 3, ng = 64 * g8;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  // A slice -> registers first (L2 hits, back before the weight stream)
  f32x4 va[RD_AG][2];
#pragma unroll
  for (int u = 0; u < RD_AG; ++u) {
    va[u][0] = z4;
    va[u][1] = z4;
    const int idx = tid + 256 * u;
    if (idx < ng) {
      const int r = idx / g8, k = k0 + (idx - r * g8) * 8;
      if (r < g.M && k < kend) {  // K % 8 == 0, 16-byte aligned rows (rd_plan): whole groups
        const float* p = g.A + (long)r * g.lda + k;
        va[u][0] = *reinterpret_cast<const f32x4*>(p);
        va[u][1] = *reinterpret_cast<const f32x4*>(p + 4);
      }
    }
  }
  // every B fragment of the slice: lane -> column (lane & 15) of block cb, k = 32s + 8(lane >> 4)
  bf16x8 vb[RD_KT][2];
  const __bf16* Bt = reinterpret_cast<const __bf16*>(g.Bt16);
#pragma unroll
  for (int s = 0; s < RD_KT; ++s)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      for (int e = 0; e < 8; ++e) vb[s][cb][e] = (__bf16)0.f;
      const int col = n0 + 32 * w + 16 * cb + (lane & 15), k = k0 + 32 * s + 8 * (lane >> 4);
      if (s < nks && col < g.N && k < kend) vb[s][cb] = *reinterpret_cast<const bf16x8*>(Bt + (long)col * g.ldbt + k);
    }
#pragma unroll
  for (int u = 0; u < RD_AG; ++u) {
    const int idx = tid + 256 * u;
    if (idx < ng) {
      const int r = idx / g8, kk = (idx - r * g8) * 8;
      bf16x8 h;
      to_bf16x8(reinterpret_cast<const float*>(&va[u][0]), h);
      *reinterpret_cast<bf16x8*>(rd_sm + r * LD + kk) = h;
    }
  }
  __syncthreads();
  f32x4 acc[4][2];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) acc[mb][0] = acc[mb][1] = z4;
  const __bf16* pa = rd_sm + (lane & 15) * LD + 8 * (lane >> 4);
#pragma unroll
  for (int s = 0; s < RD_KT; ++s) {
    if (s < nks) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(pa + 16 * mb * LD + 32 * s);
        acc[mb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, vb[s][0], acc[mb][0], 0, 0, 0);
        acc[mb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, vb[s][1], acc[mb][1], 0, 0, 0);
      }
    }
  }
  // D layout: lane -> column lane & 15, rows 4(lane >> 4) + r of each 16 x 16 block
  const bool part = g.ksplit > 1 || g.raw;
  float* P = part ? g.kpart + (long)blockIdx.z * g.M * g.N : nullptr;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int col = n0 + 32 * w + 16 * cb + (lane & 15);
    if (col >= g.N) continue;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mb + 4 * (lane >> 4) + r;
        if (row >= g.M) continue;
        if (part) P[(long)row * g.N + col] = acc[mb][cb][r];
        else epilogue_one(g, row, col, acc[mb][cb][r]);
      }
  }
}

// K split / slice of the register-direct kernel: ~one work-group per CU, slice <= 32·RD_KT
static bool rd_plan(const GemmArgs& a, int& ks, int& kslice) {
  if (a.split16 != 2 || !a.Bt16 || a.a_mode != A_DENSE || a.M > 64 || a.K < 32 || a.K % 8 || a.lda % 4 ||
      (reinterpret_cast<uintptr_t>(a.A) & 15))
    return false;
  const int nt = (a.N + RD_BN - 1) / RD_BN;
  // ~one work-group per CU (TT2_RD_TARGET work-groups), but >= 4 k-steps per slice: a small
  // product is not worth its partials
  static const int target = [] {
    const char* e = std::getenv("TT2_RD_TARGET");
    return e ? std::max(1, std::atoi(e)) : 256;
  }();
  ks = std::max(1, std::min(a.K / 128, target / std::max(nt, 1)));
  for (;;) {
    kslice = ((a.K + ks - 1) / ks + 31) / 32 * 32;
    if (kslice <= 32 * RD_KT) break;
    ++ks;
  }
  ks = (a.K + kslice - 1) / kslice;  // no empty slices
  if (ks > 1 && !a.kpart) return false;
  if (ks > 1 && (long)ks * a.M * a.N > a.kpart_floats) return false;
  return true;
}

// K split / slice of the skinny kernel: ~one work-group per CU, slice <= SK_KMAX (LDS), multiple of 32
constexpr int SK_KMAX = 608;
static bool sk_plan(const GemmArgs& a, int& ks, int& kslice) {
  if (a.split16 != 2 || !a.Bt16 || a.a_mode != A_DENSE || a.M > SK_BM || a.K < 32) return false;
  const int nt = (a.N + SK_BN - 1) / SK_BN;
  ks = std::max(1, std::min(16, 256 / std::max(nt, 1)));
  for (;;) {
    kslice = ((a.K + ks - 1) / ks + 31) / 32 * 32;
    if (kslice <= SK_KMAX) break;
    ++ks;
  }
  ks = (a.K + kslice - 1) / kslice;  // no empty slices
  if (ks > 1 && !a.kpart) return false;
  if (ks > 1 && (long)ks * a.M * a.N > a.kpart_floats) return false;
  return true;
}

template <int WMB, int WNB>
static void launch(const GemmArgs& a, bool va, bool vb, hipStream_t s) {
  dim3 grid(cdiv(a.N, 64 * WNB), cdiv(a.M, 64 * WMB), a.ksplit);
  if (va && vb) hipLaunchKernelGGL((gemm_kernel<WMB, WNB, true, true>), grid, dim3(256), 0, s, a);
  else if (va) hipLaunchKernelGGL((gemm_kernel<WMB, WNB, true, false>), grid, dim3(256), 0, s, a);
  else if (vb) hipLaunchKernelGGL((gemm_kernel<WMB, WNB, false, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((gemm_kernel<WMB, WNB, false, false>), grid, dim3(256), 0, s, a);
  TT2_HIP(hipGetLastError());
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int gemm_impl(const GemmArgs& a, hipStream_t s);

void split_weights(const float* B, int K, int N, long ldb, SplitB& out, hipStream_t s) {
  out.ldbt = (K + 7) / 8 * 8;
  const size_t n = (size_t)N * out.ldbt;
  out.hi.alloc(n * sizeof(_Float16));
  out.lo.alloc(n * sizeof(_Float16));
  hipLaunchKernelGGL(k_split_bt, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, B, K, N, ldb, out.ldbt,
                     out.hi.as<_Float16>(), out.lo.as<_Float16>());
  TT2_HIP(hipGetLastError());
}

// ---- conv1d over pre-split activation planes (gemm.h ConvX3Args) ---------------
// In the padded row layout a tap is a row shift, so with Cp the channel stride the operand is the
// overlapping-row view A[m][k] = plane[(CX_G + m - pad)·Cp + k], k = tap·Cp + c: a dense row-major
// matrix of row stride Cp over K = kw·Cp.  Same block tile, split and MFMA order as
// gemm_x3_kernel<·, 1, 2, true> (so the result matches the im2col path bit for bit when C == Cp);
// the blockIdx -> tile map keeps the N tiles of one row tile on one XCD (shared A rows in its L2);
// the planes epilogue stages the 128 x 128 output tile in LDS and writes whole 16-byte chunks.
__global__ void k_split_rows(const float* __restrict__ X, int B, int T, int C, long xs_b, _Float16* __restrict__ hi,
                             _Float16* __restrict__ lo, int Cp, long rows) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * Cp) return;
  const long r = i / Cp;
  const int c = (int)(i - r * Cp);
  const long rr = r - CX_G;
  const int Tp = T + 2 * CX_P;
  float x = 0.f;
  if (rr >= 0 && rr < (long)B * Tp && c < C) {
    const int b = (int)(rr / Tp), t = (int)(rr - (long)b * Tp) - CX_P;
    if (t >= 0 && t < T) x = X[b * xs_b + (long)t * C + c];
  }
  x *= X3_SA;
  const _Float16 h = (_Float16)x;
  hi[i] = h;
  lo[i] = (_Float16)(x - (float)h);
}

__global__ void k_split_conv_w(const float* __restrict__ W, int kw, int C, int Cp, int N, _Float16* __restrict__ hi,
                               _Float16* __restrict__ lo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int K = kw * Cp;
  if (i >= (long)N * K) return;
  const int n = (int)(i / K), k = (int)(i - (long)n * K), tap = k / Cp, c = k - tap * Cp;
  const float x = c < C ? W[((long)tap * C + c) * N + n] * X3_SB : 0.f;
  const _Float16 h = (_Float16)x;
  hi[i] = h;
  lo[i] = (_Float16)(x - (float)h);
}

// Per-column epilogue constants (bias, BN scale / shift; the identity when absent), loaded once
// per thread, and the activation as a compile-time branch of one uniform dispatch: the element
// loops are straight-line code with no loads in them.
struct CxCol {
  float b, s, h;
};
__device__ __forceinline__ CxCol cx_col(const ConvX3Args& g, int col) {
  CxCol c;
  c.b = g.bias ? g.bias[col] : 0.f;
  c.s = g.bn_scale ? g.bn_scale[col] : 1.f;
  c.h = g.bn_shift ? g.bn_shift[col] : 0.f;
  return c;
}
// tanh = 1 - 2 / (e^{2x} + 1) on v_exp_f32 + v_rcp_f32: |abs err| < 3e-7 (libm tanhf: ~10x the
// instructions, which made the 65k-element epilogue of a 256 x 256 tile cost ~20 us per layer)
__device__ __forceinline__ float cx_tanh(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * x) + 1.f); }
template <int ACT>
__device__ __forceinline__ float cx_epi(float acc, const CxCol& c) {
  float y = acc * X3_UNSCALE + c.b;
  if constexpr (ACT == ACT_RELU) y = fmaxf(y, 0.f);
  if constexpr (ACT == ACT_TANH) y = cx_tanh(y);
  y = y * c.s + c.h;
  if constexpr (ACT == ACT_BN_RELU) y = fmaxf(y, 0.f);
  return y;
}
template <class F>
__device__ __forceinline__ void cx_act(int act, F&& f) {
  if (act == ACT_TANH) f(std::integral_constant<int, ACT_TANH>{});
  else if (act == ACT_RELU) f(std::integral_constant<int, ACT_RELU>{});
  else if (act == ACT_BN_RELU) f(std::integral_constant<int, ACT_BN_RELU>{});
  else f(std::integral_constant<int, ACT_NONE>{});
}

// k-step order: 32-channel chunk major, tap minor (k0 = tap·Cp + 32·chunk), so the kw taps that
// re-read one row block (shifted by one row each) run back to back and hit L2; tap-major order
// re-streamed the A rows from MALL once per tap (~5x the unique operand bytes)
__device__ __forceinline__ int cx_k0(int kt, int kw, int Cp) {
  const int chunk = kt / kw;
  return (kt - chunk * kw) * Cp + chunk * X3_BK;
}

template <bool F32OUT>
__global__ __launch_bounds__(256, 2) void conv_x3_kernel(ConvX3Args g, int n_mt, int n_nt) {
  constexpr int BK = X3_BK, LD = X3_LD, OLD = CX_BN + 8;
  __shared__ __attribute__((aligned(16))) _Float16 sm[2][2][CX_BM + CX_BN][LD];  // [plane][buf][A rows | B cols][k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int mt = (jb / n_nt) * 8 + xcd, nt = jb - (jb / n_nt) * n_nt;
  if (mt >= n_mt) return;
  const int m0 = mt * CX_BM, n0 = nt * CX_BN;
  const int wm = wave >> 1, wn = wave & 1;
  const int am = tid >> 1, ak = (tid & 1) * 16;    // A: row am, k [ak, ak + 16)
  const int bn = tid & 127, bk = (tid >> 7) * 16;  // B: column bn, k [bk, bk + 16)
  const int pad = (g.kw - 1) >> 1;
  // split-K slice blockIdx.y of gridDim.y: k-steps [kt0, kt0 + nk)
  const int nkt = g.kw * g.Cp / BK, per = (nkt + gridDim.y - 1) / gridDim.y, kt0 = blockIdx.y * per;
  const int nk = min(nkt, kt0 + per) - kt0;
  const long aoff = (long)(CX_G + m0 + am - pad) * g.Cp + ak;
  const _Float16* pah = g.Ah + aoff;
  const _Float16* pal = g.Al + aoff;
  const bool bok = n0 + bn < g.N;
  const long boff = (long)(bok ? n0 + bn : 0) * g.ldbt + bk;
  const _Float16* pbh = g.Bh + boff;
  const _Float16* pbl = g.Bl + boff;
  f16x8 ra[2][2], rb[2][2];  // [plane][8-k half]
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  auto gload = [&](int kt) {
    const int k0 = cx_k0(kt0 + kt, g.kw, g.Cp);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ra[0][h] = *reinterpret_cast<const f16x8*>(pah + k0 + 8 * h);
      ra[1][h] = *reinterpret_cast<const f16x8*>(pal + k0 + 8 * h);
      if (bok) {
        rb[0][h] = *reinterpret_cast<const f16x8*>(pbh + k0 + 8 * h);
        rb[1][h] = *reinterpret_cast<const f16x8*>(pbl + k0 + 8 * h);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rb[0][h][e] = rb[1][h][e] = (_Float16)0.f;
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        *reinterpret_cast<f16x8*>(&sm[p][buf][am][ak + 8 * h]) = ra[p][h];
        *reinterpret_cast<f16x8*>(&sm[p][buf][CX_BM + bn][bk + 8 * h]) = rb[p][h];
      }
  };
  if (nk > 0) {  // an uneven K split can leave a slice empty: it still writes its zero partial
    gload(0);
    sstore(0);
  }
  __syncthreads();
  const int r = lane & 31, h8 = (lane >> 5) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int s16 = 0; s16 < BK; s16 += 16) {
      f16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = *reinterpret_cast<const f16x8*>(&sm[0][cur][wm * 64 + i * 32 + r][s16 + h8]);
        al[i] = *reinterpret_cast<const f16x8*>(&sm[1][cur][wm * 64 + i * 32 + r][s16 + h8]);
        bh[i] = *reinterpret_cast<const f16x8*>(&sm[0][cur][CX_BM + wn * 64 + i * 32 + r][s16 + h8]);
        bl[i] = *reinterpret_cast<const f16x8*>(&sm[1][cur][CX_BM + wn * 64 + i * 32 + r][s16 + h8]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  // epilogue: padded row m -> (b, t); pad rows (and rows past B·Tp) are not frames
  const int Tp = g.T + 2 * CX_P;
  const long mrows = (long)g.B * Tp;
  if (g.ks > 1) {  // raw partials of this K slice (padded rows), reduced by k_cx_reduce
    float* P = g.part + (long)blockIdx.y * mrows * g.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const long m = m0 + wm * 64 + i * 32 + 4 * (lane >> 5) + (q & 3) + 8 * (q >> 2);
          if (m < mrows && col < g.N) P[m * g.N + col] = acc[i][j][q];
        }
      }
    return;
  }
  _Float16* ot = &sm[0][0][0][0];  // [plane][128][OLD] output tile (the loop's last barrier freed LDS)
  int orow[2][16];                 // output row b·T + t of (i, q), -1 for pad / tail rows
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int mb0 = m0 + wm * 64 + i * 32 + 4 * (lane >> 5), b0 = mb0 / Tp, t00 = mb0 - b0 * Tp;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rq = (q & 3) + 8 * (q >> 2);
      int t = t00 + rq, b = b0;
      while (t >= Tp) { t -= Tp; ++b; }
      const bool frame = (long)mb0 + rq < mrows && t >= CX_P && t < CX_P + g.T;
      orow[i][q] = frame ? b * g.T + (t - CX_P) : -1;
    }
  }
  CxCol cc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) cc[j] = cx_col(g, min(n0 + wn * 64 + j * 32 + (lane & 31), g.N - 1));
  if constexpr (F32OUT) {
    float res[2][2][16];  // residual operands, all loads issued before any use
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int col = min(n0 + wn * 64 + j * 32 + (lane & 31), g.N - 1);
          res[i][j][q] = g.residual ? g.residual[(long)max(orow[i][q], 0) * g.ldr + col] : 0.f;
        }
    cx_act(g.act, [&](auto A) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            float y = res[i][j][q] + cx_epi<decltype(A)::value>(acc[i][j][q], cc[j]);
            if (g.clip) y = fminf(fmaxf(y, g.clip_lo), g.clip_hi);
            if (orow[i][q] >= 0 && col < g.N) g.Cout[(long)orow[i][q] * g.ldc + col] = y;
          }
        }
    });
  } else {
    cx_act(g.act, [&](auto A) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rl = wm * 64 + i * 32 + 4 * (lane >> 5) + (q & 3) + 8 * (q >> 2);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int cl = wn * 64 + j * 32 + (lane & 31);
            const float y = orow[i][q] >= 0 ? cx_epi<decltype(A)::value>(acc[i][j][q], cc[j]) * X3_SA : 0.f;
            const _Float16 hv = (_Float16)y;
            ot[rl * OLD + cl] = hv;
            ot[CX_BM * OLD + rl * OLD + cl] = (_Float16)(y - (float)hv);
          }
        }
    });
  }
  if constexpr (!F32OUT) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = tid + 256 * u, p = idx >> 11, rl = (idx >> 4) & 127, ch = idx & 15;
      const long m = (long)m0 + rl;
      if (m < mrows)
        *reinterpret_cast<f16x8*>((p ? g.Ol : g.Oh) + (CX_G + m) * g.N + n0 + 8 * ch) =
            *reinterpret_cast<const f16x8*>(ot + p * CX_BM * OLD + rl * OLD + 8 * ch);
    }
  }
}

// Wide form for planes output with N % 256 == 0 (the 512-channel Postnet layers): 256 x 256 tile,
// 8 waves (2 along M x 4 along N, wave tile 128 x 64 = 4 x 2 accumulators), one work-group per CU.
// Operands are staged by LDS-DMA (global_load_lds, 16 B per lane) into a lane-linear image of
// 64-byte rows (32 k of one operand plane); the 16-byte chunks of row R sit XOR-swizzled by
// (R >> 2) & 3, applied on the DMA source address and on the fragment read, so the 16 lanes of a
// ds_read_b128 group hit 16 distinct bank slots.  Two stages: the next k-step's DMA is issued
// before the current step's 48 MFMAs per wave and retired (vmcnt 0 + barrier) after them.
constexpr int CXW_BM = 256, CXW_BN = 256, CXW_PLANE = 256 * X3_BK, CXW_OLD = CXW_BN + 8;
constexpr int CXW_LDS = (2 * 4 * CXW_PLANE > CXW_BM * CXW_OLD) ? 2 * 4 * CXW_PLANE : CXW_BM * CXW_OLD;  // halfs

template <int ACT>
__device__ __forceinline__ void cxw_apply(f32x16 (&acc)[4][2], const unsigned (&fm)[4], const CxCol (&cc)[2]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j][q] = ((fm[i] >> q) & 1u) ? cx_epi<ACT>(acc[i][j][q], cc[j]) * X3_SA : 0.f;
}

template <int ACT, bool SPLIT = false, bool F32OUT = false>
__global__ __launch_bounds__(512, 1) void conv_x3w_kernel(ConvX3Args g, int n_mt, int n_nt) {
  __shared__ __attribute__((aligned(16))) _Float16 sm[CXW_LDS];  // [stage][A hi, A lo, B hi, B lo][256][32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int mt = (jb / n_nt) * 8 + xcd, nt = jb - (jb / n_nt) * n_nt;
  if (mt >= n_mt) return;
  const int m0 = mt * CXW_BM, n0 = nt * CXW_BN;
  const int wm = wave >> 2, wn = wave & 3;
  const int pad = (g.kw - 1) >> 1;
  // DMA pieces: wave w fills rows [32w, 32w + 32) of every plane as two 16-row pieces; lane l lands
  // at row (l >> 2), physical chunk l & 3, and fetches logical chunk (l & 3) ^ ((l >> 4) & 3)
  const int srow = 32 * wave + (lane >> 2), sc = (lane & 3) ^ ((lane >> 4) & 3);
  const _Float16 *ga[2][2], *gb[2][2];  // [plane][piece]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long ao = (long)(CX_G + m0 + srow + 16 * i - pad) * g.Cp + 8 * sc;
    const long bo = (long)(n0 + srow + 16 * i) * g.ldbt + 8 * sc;
    ga[0][i] = g.Ah + ao;
    ga[1][i] = g.Al + ao;
    gb[0][i] = g.Bh + bo;
    gb[1][i] = g.Bl + bo;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr;
  auto stage = [&](int kt, int buf) {
    const int k0 = cx_k0(kt, g.kw, g.Cp);
    _Float16* base = sm + buf * 4 * CXW_PLANE + 32 * wave * X3_BK;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        __builtin_amdgcn_global_load_lds(ga[p][i] + k0, (lds_ptr)(base + p * CXW_PLANE + 16 * i * X3_BK), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(gb[p][i] + k0, (lds_ptr)(base + (2 + p) * CXW_PLANE + 16 * i * X3_BK), 16, 0, 0);
      }
  };
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  // K split over blockIdx.y (ConvX3Args::ks): k-steps [kt0, kt0 + nk)
  const int nkt = g.kw * g.Cp / X3_BK, per = SPLIT ? (nkt + gridDim.y - 1) / gridDim.y : nkt;
  const int kt0 = SPLIT ? blockIdx.y * per : 0, nk = SPLIT ? min(nkt, kt0 + per) - kt0 : nkt;
  if (nk > 0) stage(kt0, 0);  // an empty K slice (uneven split) reads nothing, writes zeros
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int r = lane & 31, hl = lane >> 5, sw = (r >> 2) & 3;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt0 + kt + 1, cur ^ 1);
    const _Float16* S = sm + cur * 4 * CXW_PLANE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int off = r * X3_BK + 8 * ((2 * s + hl) ^ sw);
      f16x8 bh[2], bl[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bh[j] = *reinterpret_cast<const f16x8*>(S + 2 * CXW_PLANE + (wn * 64 + j * 32) * X3_BK + off);
        bl[j] = *reinterpret_cast<const f16x8*>(S + 3 * CXW_PLANE + (wn * 64 + j * 32) * X3_BK + off);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f16x8 ah = *reinterpret_cast<const f16x8*>(S + (wm * 128 + i * 32) * X3_BK + off);
        const f16x8 al = *reinterpret_cast<const f16x8*>(S + CXW_PLANE + (wm * 128 + i * 32) * X3_BK + off);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue: y·2^4 in place (pad rows and rows past B·Tp -> 0), then each plane through LDS
  const int Tp = g.T + 2 * CX_P;
  const long mrows = (long)g.B * Tp;
  if constexpr (SPLIT) {  // raw partials of this K slice (padded rows), combined by k_cx_reduce
    float* P = g.part + (long)blockIdx.y * mrows * g.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + r;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const long m = m0 + wm * 128 + i * 32 + 4 * hl + (q & 3) + 8 * (q >> 2);
          if (m < mrows) P[m * g.N + col] = acc[i][j][q];
        }
      }
    return;
  }
  if constexpr (F32OUT) {  // fp32 frame rows b·T + t (no activation / BN / residual: the projections)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mb0 = m0 + wm * 128 + i * 32 + 4 * hl, b0 = mb0 / Tp, t00 = mb0 - b0 * Tp;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + r;
        const float bias = g.bias ? g.bias[col] : 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rq = (q & 3) + 8 * (q >> 2);
          int t = t00 + rq, b = b0;
          while (t >= Tp) { t -= Tp; ++b; }
          if (b < g.B && t >= CX_P && t < CX_P + g.T)
            g.Cout[((long)b * g.T + t - CX_P) * g.ldc + col] = acc[i][j][q] * X3_UNSCALE + bias;
        }
      }
    }
    return;
  }
  unsigned fm[4] = {0u, 0u, 0u, 0u};  // frame bit of (i, q)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int mb0 = m0 + wm * 128 + i * 32 + 4 * hl, b0 = mb0 / Tp, t00 = mb0 - b0 * Tp;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rq = (q & 3) + 8 * (q >> 2);
      int t = t00 + rq;
      while (t >= Tp) t -= Tp;
      if ((long)mb0 + rq < mrows && t >= CX_P && t < CX_P + g.T) fm[i] |= 1u << q;
    }
  }
  CxCol cc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) cc[j] = cx_col(g, n0 + wn * 64 + j * 32 + r);
  cxw_apply<ACT>(acc, fm, cc);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if (p) __syncthreads();  // the hi plane's copy-out has read the tile
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int rl = wm * 128 + i * 32 + 4 * hl + (q & 3) + 8 * (q >> 2);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float v = acc[i][j][q];
          const _Float16 hv = (_Float16)v;
          sm[rl * CXW_OLD + wn * 64 + j * 32 + r] = p ? (_Float16)(v - (float)hv) : hv;
        }
      }
    __syncthreads();
    _Float16* O = p ? g.Ol : g.Oh;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = tid + 512 * u, rl = idx >> 5, ch = idx & 31;
      const long m = (long)m0 + rl;
      if (m < mrows)
        *reinterpret_cast<f16x8*>(O + (CX_G + m) * g.N + n0 + 8 * ch) =
            *reinterpret_cast<const f16x8*>(sm + rl * CXW_OLD + 8 * ch);
    }
  }
}

// split-K combine of conv_x3_kernel partials: 4 consecutive channels of one padded row per thread,
// the same epilogue as the kernels (planes with zero pad rows, or fp32 frame rows + residual / clip)
template <int ACT>
__global__ __launch_bounds__(256) void k_cx_reduce(ConvX3Args g, long mrows) {
  const int n4 = g.N >> 2;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= mrows * n4) return;
  const long m = i / n4;
  const int c = (int)(i - m * n4) * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < g.ks; ++z) acc += *reinterpret_cast<const f32x4*>(g.part + ((long)z * mrows + m) * g.N + c);
  const int Tp = g.T + 2 * CX_P, b = (int)(m / Tp), t = (int)(m - (long)b * Tp) - CX_P;
  const bool frame = t >= 0 && t < g.T;
  float y[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) y[e] = frame ? cx_epi<ACT>(acc[e], cx_col(g, c + e)) : 0.f;
  if (g.Oh) {
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    f16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = y[e] * X3_SA;
      h[e] = (_Float16)x;
      l[e] = (_Float16)(x - (float)h[e]);
    }
    *reinterpret_cast<f16x4*>(g.Oh + (CX_G + m) * g.N + c) = h;
    *reinterpret_cast<f16x4*>(g.Ol + (CX_G + m) * g.N + c) = l;
  } else if (frame) {
    const long orow = (long)b * g.T + t;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = y[e] + (g.residual ? g.residual[orow * g.ldr + c + e] : 0.f);
      if (g.clip) v = fminf(fmaxf(v, g.clip_lo), g.clip_hi);
      g.Cout[orow * g.ldc + c + e] = v;
    }
  }
}

void split_rows(const float* X, int B, int T, int C, long xs_b, _Float16* hi, _Float16* lo, int Cp, hipStream_t s) {
  const long rows = cx_rows(B, T), n = rows * Cp;
  hipLaunchKernelGGL(k_split_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, X, B, T, C, xs_b, hi, lo, Cp, rows);
  TT2_HIP(hipGetLastError());
}

void split_conv_weights(const float* W, int kw, int C, int Cp, int N, SplitB& out, hipStream_t s) {
  out.ldbt = (long)kw * Cp;
  const size_t n = (size_t)N * out.ldbt;
  out.hi.alloc(n * sizeof(_Float16));
  out.lo.alloc(n * sizeof(_Float16));
  hipLaunchKernelGGL(k_split_conv_w, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, kw, C, Cp, N,
                     out.hi.as<_Float16>(), out.lo.as<_Float16>());
  TT2_HIP(hipGetLastError());
}

void conv_x3(const ConvX3Args& a, hipStream_t s) {
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  TT2_CHECK(a.B > 0 && a.T > 0 && a.N > 0 && a.Cp > 0 && a.Cp % X3_BK == 0 && (a.kw & 1) && a.kw <= 2 * CX_P + 1,
            TT2_ERR_SHAPE_MISMATCH, "conv_x3: needs Cp % 32 == 0 and an odd kw <= 5");
  TT2_CHECK(a.Ah && a.Al && a.Bh && a.Bl && a16(a.Ah) && a16(a.Al) && a16(a.Bh) && a16(a.Bl) &&
                a.ldbt >= (long)a.kw * a.Cp && a.ldbt % 8 == 0,
            TT2_ERR_INVALID_ARG, "conv_x3: operand planes missing or misaligned");
  TT2_CHECK((a.Oh != nullptr) != (a.Cout != nullptr), TT2_ERR_INVALID_ARG, "conv_x3: exactly one output");
  TT2_CHECK(!a.Oh || (a.Ol && a.N % CX_BN == 0 && a16(a.Oh) && a16(a.Ol)), TT2_ERR_INVALID_ARG,
            "conv_x3: planes output needs N % 128 == 0 and aligned planes");
  const char* ew = std::getenv("TT2_CX_WIDE");  // 0: the 128 x 128 register-staged kernel for every layer
  const bool wide = !ew || std::atoi(ew) != 0;
  if (a.ks > 1) {  // split K over blockIdx.y + one combine launch
    const long mrows = (long)a.B * (a.T + 2 * CX_P);
    TT2_CHECK(a.part && a.N % 4 == 0 && (long)a.ks * mrows * a.N <= a.part_floats && a.ks <= a.kw * a.Cp / X3_BK,
              TT2_ERR_INVALID_ARG, "conv_x3: split-K needs part >= ks x rows x N floats, N % 4 == 0");
    const char* ewk = std::getenv("TT2_CX_WIDE_SPLIT");  // 0: the 128 x 128 kernel for the K-split layers
    if (a.N % CXW_BN == 0 && (!ewk || std::atoi(ewk) != 0)) {
      const int n_mt = cdiv(a.B * (a.T + 2 * CX_P), CXW_BM), n_nt = a.N / CXW_BN;
      hipLaunchKernelGGL((conv_x3w_kernel<ACT_NONE, true>), dim3((unsigned)(cdiv(n_mt, 8) * 8 * n_nt), (unsigned)a.ks),
                         dim3(512), 0, s, a, n_mt, n_nt);
    } else {
      const int n_mt = cdiv(a.B * (a.T + 2 * CX_P), CX_BM), n_nt = cdiv(a.N, CX_BN);
      const dim3 grid((unsigned)(cdiv(n_mt, 8) * 8 * n_nt), (unsigned)a.ks);
      hipLaunchKernelGGL(conv_x3_kernel<false>, grid, dim3(256), 0, s, a, n_mt, n_nt);
    }
    TT2_HIP(hipGetLastError());
    const dim3 rg((unsigned)((mrows * (a.N / 4) + 255) / 256));
    if (a.act == ACT_TANH) hipLaunchKernelGGL(k_cx_reduce<ACT_TANH>, rg, dim3(256), 0, s, a, mrows);
    else if (a.act == ACT_RELU) hipLaunchKernelGGL(k_cx_reduce<ACT_RELU>, rg, dim3(256), 0, s, a, mrows);
    else if (a.act == ACT_BN_RELU) hipLaunchKernelGGL(k_cx_reduce<ACT_BN_RELU>, rg, dim3(256), 0, s, a, mrows);
    else hipLaunchKernelGGL(k_cx_reduce<ACT_NONE>, rg, dim3(256), 0, s, a, mrows);
    TT2_HIP(hipGetLastError());
    return;
  }
  if (wide && a.Cout && a.N % CXW_BN == 0 && a.act == ACT_NONE && !a.bn_scale && !a.residual && !a.clip) {
    const int n_mt = cdiv(a.B * (a.T + 2 * CX_P), CXW_BM), n_nt = a.N / CXW_BN;
    hipLaunchKernelGGL((conv_x3w_kernel<ACT_NONE, false, true>), dim3((unsigned)(cdiv(n_mt, 8) * 8 * n_nt)), dim3(512),
                       0, s, a, n_mt, n_nt);
    TT2_HIP(hipGetLastError());
    return;
  }
  if (wide && a.Oh && a.N % CXW_BN == 0) {
    const int n_mt = cdiv(a.B * (a.T + 2 * CX_P), CXW_BM), n_nt = a.N / CXW_BN;
    const dim3 grid((unsigned)(cdiv(n_mt, 8) * 8 * n_nt));
    if (a.act == ACT_TANH) hipLaunchKernelGGL(conv_x3w_kernel<ACT_TANH>, grid, dim3(512), 0, s, a, n_mt, n_nt);
    else if (a.act == ACT_RELU) hipLaunchKernelGGL(conv_x3w_kernel<ACT_RELU>, grid, dim3(512), 0, s, a, n_mt, n_nt);
    else if (a.act == ACT_BN_RELU) hipLaunchKernelGGL(conv_x3w_kernel<ACT_BN_RELU>, grid, dim3(512), 0, s, a, n_mt, n_nt);
    else hipLaunchKernelGGL(conv_x3w_kernel<ACT_NONE>, grid, dim3(512), 0, s, a, n_mt, n_nt);
    TT2_HIP(hipGetLastError());
    return;
  }
  const int n_mt = cdiv(a.B * (a.T + 2 * CX_P), CX_BM), n_nt = cdiv(a.N, CX_BN);
  const dim3 grid((unsigned)(cdiv(n_mt, 8) * 8 * n_nt));
  if (a.Cout) hipLaunchKernelGGL(conv_x3_kernel<true>, grid, dim3(256), 0, s, a, n_mt, n_nt);
  else hipLaunchKernelGGL(conv_x3_kernel<false>, grid, dim3(256), 0, s, a, n_mt, n_nt);
  TT2_HIP(hipGetLastError());
}

// ---- large bf16 product over K-contiguous operands (gemm.h gemm_bf16_kc) ----------------------
constexpr int KC_BM = 256, KC_BN = 256, KC_BK = 64, KC_PLANE = 256 * KC_BK;  // bf16 per operand per stage

// A[M][K] fp32 (row stride lda) -> a16[Mp][Kp] bf16, zero padded
__global__ void k_kc_pad(const float* __restrict__ A, int M, int K, long lda, __bf16* __restrict__ out, int Kp,
                         long n4) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long e = i * 4, r = e / Kp;
    const int k = (int)(e - r * Kp);
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (__bf16)((r < M && k + q < K) ? A[r * lda + k + q] : 0.f);
    *reinterpret_cast<bf16x4*>(out + e) = o;
  }
}

// B[K][N] fp32 (row stride ldb) -> b16[Np][Kp] bf16 (transposed, zero padded): 64 x 64 tiles through
// LDS, 256-byte coalesced row reads, 128-byte coalesced transposed row writes
__global__ __launch_bounds__(256) void k_kc_tr(const float* __restrict__ B, int K, int N, long ldb,
                                               __bf16* __restrict__ out, int Kp) {
  __shared__ float t[64][65];
  const int k0 = blockIdx.x * 64, n0 = blockIdx.y * 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int kk = ty; kk < 64; kk += 4)
    t[kk][tx] = (k0 + kk < K && n0 + tx < N) ? B[(long)(k0 + kk) * ldb + n0 + tx] : 0.f;
  __syncthreads();
#pragma unroll 4
  for (int nn = ty; nn < 64; nn += 4) out[(long)(n0 + nn) * Kp + k0 + tx] = (__bf16)t[tx][nn];
}

// the conv weight gradient's transposed im2col (KcConvA) -> a16[Mp][Kp] bf16: 64 (frames) x 64 (tap,
// channel) tiles; reads are 256-byte runs of one frame's channels, writes 128-byte runs of frames
__global__ __launch_bounds__(256) void k_kc_im2col(KcConvA cv, __bf16* __restrict__ out, int Kp) {
  __shared__ float t[64][65];
  const int k0 = blockIdx.x * 64, n0 = blockIdx.y * 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int K = cv.B * cv.T, M = cv.kw * cv.C;
  const int n = n0 + tx, tap = n / cv.C, c = n - tap * cv.C;
#pragma unroll 4
  for (int kk = ty; kk < 64; kk += 4) {
    const int m = k0 + kk;
    float v = 0.f;
    if (m < K && n < M) {
      const int b = m / cv.T, ts = m - b * cv.T + tap - cv.pad;
      if (ts >= 0 && ts < cv.T) v = cv.x[(long)b * cv.xs_b + (long)ts * cv.xs_t + c];
    }
    t[kk][tx] = v;
  }
  __syncthreads();
#pragma unroll 4
  for (int nn = ty; nn < 64; nn += 4) out[(long)(n0 + nn) * Kp + k0 + tx] = (__bf16)t[tx][nn];
}

// 256 x 256 tile, 8 waves (2 x 4, wave tile 128 x 64 = 4 x 2 v_mfma_f32_32x32x16_bf16 accumulators),
// 64-deep k-steps staged by LDS-DMA into 128-byte rows whose 16-byte chunks sit XOR-swizzled by
// (row >> 1) & 7 (source address and fragment read), two stages; K split over blockIdx.y
template <int ACT>
__global__ __launch_bounds__(512, 1) void k_gemm_kc(const __bf16* __restrict__ A, long lda,
                                                    const __bf16* __restrict__ Bt, long ldb, int Kp, int M, int N,
                                                    float* __restrict__ C, long ldc, float* __restrict__ part,
                                                    int n_mt, int n_nt, KcEpi ep) {
  __shared__ __attribute__((aligned(16))) __bf16 sm[2 * 2 * KC_PLANE];  // [stage][A, B][256][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int mt = (jb / n_nt) * 8 + xcd, nt = jb - (jb / n_nt) * n_nt;
  if (mt >= n_mt) return;
  const int m0 = mt * KC_BM, n0 = nt * KC_BN;
  const int wm = wave >> 2, wn = wave & 3;
  const int nkt = Kp / KC_BK, per = (nkt + gridDim.y - 1) / gridDim.y, kt0 = blockIdx.y * per;
  const int nk = min(nkt, kt0 + per) - kt0;
  // DMA pieces: 8 rows x 128 B; wave w fills pieces 4w .. 4w+3 of each operand; lane l lands at row
  // 8p + (l >> 3), physical chunk l & 7, and fetches logical chunk (l & 7) ^ ((row >> 1) & 7)
  const __bf16 *ga[4], *gb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
    ga[i] = A + (long)(m0 + row) * lda + 8 * c + (long)kt0 * KC_BK;
    gb[i] = Bt + (long)(n0 + row) * ldb + 8 * c + (long)kt0 * KC_BK;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr;
  auto stage = [&](int kt, int buf) {
    const int k0 = kt * KC_BK;
    __bf16* base = sm + buf * 2 * KC_PLANE + 8 * 4 * wave * KC_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds(ga[i] + k0, (lds_ptr)(base + 8 * i * KC_BK), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(gb[i] + k0, (lds_ptr)(base + KC_PLANE + 8 * i * KC_BK), 16, 0, 0);
    }
  };
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  if (nk > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int r = lane & 31, hl = lane >> 5, sw = (r >> 1) & 7;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const __bf16* S = sm + cur * 2 * KC_PLANE;
#pragma unroll
    for (int sl = 0; sl < KC_BK / 16; ++sl) {
      const int off = r * KC_BK + 8 * ((2 * sl + hl) ^ sw);
      bf16x8 b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const bf16x8*>(S + KC_PLANE + (wn * 64 + j * 32) * KC_BK + off);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(S + (wm * 128 + i * 32) * KC_BK + off);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[j], acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (ep.T > 0) {  // conv over padded planes: padded row -> frame (b, t); act(acc + bias) -> C rows b·T + t
    const int Tp = ep.T + 2 * CX_P;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mb0 = m0 + wm * 128 + i * 32 + 4 * hl, b0 = mb0 / Tp, t00 = mb0 - b0 * Tp;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + r;
        const float bias = (ep.bias && col < N) ? ep.bias[col] : 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rq = (q & 3) + 8 * (q >> 2);
          int t = t00 + rq, b = b0;
          while (t >= Tp) { t -= Tp; ++b; }
          float y = acc[i][j][q] + bias;
          if constexpr (ACT == ACT_TANH) y = cx_tanh(y);
          if constexpr (ACT == ACT_RELU) y = fmaxf(y, 0.f);
          if (b < ep.B && t >= CX_P && t < CX_P + ep.T && col < N) C[((long)b * ep.T + t - CX_P) * ldc + col] = y;
        }
      }
    }
    return;
  }
  float* out = part ? part + (long)blockIdx.y * M * N : C;
  const long ld = part ? N : ldc;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + r;
      if (col >= N) continue;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = m0 + wm * 128 + i * 32 + 4 * hl + (q & 3) + 8 * (q >> 2);
        if (row < M) out[(long)row * ld + col] = acc[i][j][q];
      }
    }
}

void conv_bf16_planes(const __bf16* planes, int Cp, int B, int T, int kw, const __bf16* Bt, long ldbt, int N,
                      const float* bias, int act, float* out, long ldo, hipStream_t s) {
  TT2_CHECK(Cp % KC_BK == 0 && (kw & 1) && kw <= 2 * CX_P + 1 && ldbt >= (long)kw * Cp, TT2_ERR_SHAPE_MISMATCH,
            "conv_bf16_planes: needs Cp % 64 == 0, odd kw <= 5");
  const int Mr = B * (T + 2 * CX_P), n_mt = cdiv(Mr, KC_BM), n_nt = cdiv(N, KC_BN);
  KcEpi ep;
  ep.T = T; ep.B = B; ep.bias = bias;
  const __bf16* A = planes + (long)(CX_G - (kw - 1) / 2) * Cp;  // the overlapping-row view, row stride Cp
  const dim3 grid((unsigned)(cdiv(n_mt, 8) * 8 * n_nt));
  if (act == ACT_TANH)
    hipLaunchKernelGGL(k_gemm_kc<ACT_TANH>, grid, dim3(512), 0, s, A, (long)Cp, Bt, ldbt, kw * Cp, Mr, N, out, ldo,
                       nullptr, n_mt, n_nt, ep);
  else if (act == ACT_RELU)
    hipLaunchKernelGGL(k_gemm_kc<ACT_RELU>, grid, dim3(512), 0, s, A, (long)Cp, Bt, ldbt, kw * Cp, Mr, N, out, ldo,
                       nullptr, n_mt, n_nt, ep);
  else
    hipLaunchKernelGGL(k_gemm_kc<ACT_NONE>, grid, dim3(512), 0, s, A, (long)Cp, Bt, ldbt, kw * Cp, Mr, N, out, ldo,
                       nullptr, n_mt, n_nt, ep);
  TT2_HIP(hipGetLastError());
}

void kc_transpose_bf16(const float* B, int K, int N, long ldb, __bf16* out, int Kp, int Np, hipStream_t s) {
  TT2_CHECK(Kp % 64 == 0 && Np % 64 == 0 && Kp >= K && Np >= N, TT2_ERR_SHAPE_MISMATCH, "kc_transpose_bf16: padding");
  hipLaunchKernelGGL(k_kc_tr, dim3(Kp / 64, Np / 64), dim3(256), 0, s, B, K, N, ldb, out, Kp);
  TT2_HIP(hipGetLastError());
}

// the K split of one gemm_bf16_kc product: ks work-groups per tile over per k-steps each
static void kc_split(int M, int N, int K, int* ks_out, int* per_out) {
  const int n_mt = cdiv(M, KC_BM), n_nt = cdiv(N, KC_BN), tiles = n_mt * n_nt;
  const int nkt = cdiv(K, KC_BK);
  // K split: one work-group per CU, so the time is ~ rounds x k-steps per work-group, rounds =
  // ceil(tiles·ks / 256); plus the combine's partial traffic (ks x M x N fp32 written + read, ~9 MB
  // per k-step time of ~1.8 us at 5 TB/s): the cheapest ks <= 32 with >= 16 k-steps each and all
  // work-groups in one round (measured: 144 tiles x 7 splits over 4 rounds ran each k-step at twice
  // the time of 144 unsplit tiles -- the splits' disjoint K ranges share nothing in L2 / MALL)
  int ks = 1;
  double best = 1e30;
  for (int k = 1; k <= 32 && (k == 1 || (nkt / k >= 16 && tiles * k <= 256)); ++k) {
    const int per_k = cdiv(nkt, k), kk = cdiv(nkt, per_k);
    const double cost = (double)cdiv(tiles * kk, 256) * per_k + (kk > 1 ? kk * (double)M * N * 8 / 9e6 : 0.0);
    if (cost < best - 1e-9) { best = cost; ks = kk; }
  }
  const int per = cdiv(nkt, ks);
  ks = cdiv(nkt, per);  // no empty slices
  *ks_out = ks;
  *per_out = per;
}

void gemm_bf16_kc_bt_dims(int M, int N, int K, long* Np, long* Kp) {
  int ks, per;
  kc_split(M, N, K, &ks, &per);
  *Np = (long)cdiv(N, KC_BN) * KC_BN;
  *Kp = (long)per * ks * KC_BK;
}

void gemm_bf16_kc(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C, long ldc,
                  DevBuf& a16, DevBuf& b16, DevBuf& part, hipStream_t s, bool a_kmajor, const KcConvA* conv,
                  const __bf16* bt_pre, const __bf16* a_pre) {
  TT2_CHECK(M > 0 && N > 0 && K > 0, TT2_ERR_SHAPE_MISMATCH, "gemm_bf16_kc: empty problem");
  const int n_mt = cdiv(M, KC_BM), n_nt = cdiv(N, KC_BN);
  const int nkt = cdiv(K, KC_BK);
  int ks, per;
  kc_split(M, N, K, &ks, &per);
  (void)nkt;
  const int Kp = per * ks * KC_BK, Mp = n_mt * KC_BM, Np = n_nt * KC_BN;
  const size_t na = a_pre ? 0 : (size_t)Mp * Kp * 2, nb = bt_pre ? 0 : (size_t)Np * Kp * 2, np = ks > 1 ? (size_t)ks * M * N * 4 : 0;
  if (a16.bytes < na) a16.alloc(na);  // growth frees the old buffer (device-synchronising hipFree)
  if (b16.bytes < nb) b16.alloc(nb);
  if (part.bytes < np) part.alloc(np);
  __bf16* a = a_pre ? const_cast<__bf16*>(a_pre) : reinterpret_cast<__bf16*>(a16.p);
  const __bf16* b = bt_pre ? bt_pre : reinterpret_cast<__bf16*>(b16.p);
  const long n4 = (long)Mp * Kp / 4;
  if (a_pre) {
    // the caller staged A as [Mp][Kp] bf16 itself
  } else if (conv) {
    TT2_CHECK(conv->kw * conv->C == M && conv->B * conv->T == K, TT2_ERR_SHAPE_MISMATCH, "gemm_bf16_kc: conv shape");
    hipLaunchKernelGGL(k_kc_im2col, dim3(Kp / 64, Mp / 64), dim3(256), 0, s, *conv, a, Kp);
  } else if (a_kmajor) hipLaunchKernelGGL(k_kc_tr, dim3(Kp / 64, Mp / 64), dim3(256), 0, s, A, K, M, lda, a, Kp);
  else hipLaunchKernelGGL(k_kc_pad, dim3((unsigned)std::min<long>((n4 + 255) / 256, 8192)), dim3(256), 0, s, A, M, K,
                          lda, a, Kp, n4);
  if (!bt_pre) hipLaunchKernelGGL(k_kc_tr, dim3(Kp / 64, Np / 64), dim3(256), 0, s, B, K, N, ldb, const_cast<__bf16*>(b), Kp);
  TT2_HIP(hipGetLastError());
  float* pp = ks > 1 ? reinterpret_cast<float*>(part.p) : nullptr;
  hipLaunchKernelGGL(k_gemm_kc<ACT_NONE>, dim3((unsigned)(cdiv(n_mt, 8) * 8 * n_nt), (unsigned)ks), dim3(512), 0, s, a,
                     (long)Kp, b, (long)Kp, Kp, M, N, C, ldc, pp, n_mt, n_nt, KcEpi());
  TT2_HIP(hipGetLastError());
  if (ks > 1) {
    GemmArgs g;
    g.M = M; g.N = N; g.kpart = pp; g.ksplit = ks; g.Cout = C; g.ldc = ldc;
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(((long)M * N + 1023) / 1024)), dim3(256), 0, s, g);
    TT2_HIP(hipGetLastError());
  }
}

int gemm_raw(const GemmArgs& a, hipStream_t s) {
  TT2_CHECK(a.kpart, TT2_ERR_INVALID_ARG, "gemm_raw: kpart required");
  GemmArgs g = a;
  g.raw = 1;
  return gemm_impl(g, s);
}

void gemm(const GemmArgs& a, hipStream_t s) {
  GemmArgs g = a;
  g.raw = 0;
  (void)gemm_impl(g, s);
}

int gemm_impl(const GemmArgs& a, hipStream_t s) {
  TT2_CHECK(a.M > 0 && a.N > 0 && a.K > 0, TT2_ERR_SHAPE_MISMATCH, "gemm: empty problem");
  bool va = al16(a.A);
  if (a.a_mode == A_DENSE) va = va && (a.lda % 4 == 0);
  else if (a.a_mode == A_CONV1D) va = va && (a.C % 4 == 0) && (a.xs_t % 4 == 0) && (a.xs_b % 4 == 0);
  else va = va && (a.C % 4 == 0);
  if (a.split16) {
    TT2_CHECK(!a.Bt16 || (al16(a.Bt16) && a.ldbt % 8 == 0 && (a.split16 == 2 || (a.Bt16lo && al16(a.Bt16lo)))),
              TT2_ERR_INVALID_ARG, "gemm: Bt16 needs 16-byte alignment, ldbt % 8 == 0 (and Bt16lo for split16 == 1)");
    int sks = 0, skl = 0;
    static const int sk_mode = [] {  // TT2_GEMM_SKINNY: 2 (default) = register-direct kernel, 1 =
      const char* e = std::getenv("TT2_GEMM_SKINNY");  // LDS-staged skinny kernel, 0 = gemm_x3_kernel
      return e ? std::atoi(e) : 2;                     // (A/B: DESIGN §5.6)
    }();
    if (sk_mode == 2 && rd_plan(a, sks, skl)) {
      GemmArgs g = a;
      g.ksplit = sks;
      static bool rd_attr = false;
      if (!rd_attr) {
        TT2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_rd_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)rd_lds_bytes(32 * RD_KT)));
        rd_attr = true;
      }
      dim3 grid(cdiv(a.N, RD_BN), 1, sks);
      hipLaunchKernelGGL(gemm_rd_kernel, grid, dim3(256), rd_lds_bytes(skl), s, g, skl);
      TT2_HIP(hipGetLastError());
      if (sks > 1 && !g.raw) {
        hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(((long)a.M * a.N + 1023) / 1024)), dim3(256), 0, s, g);
        TT2_HIP(hipGetLastError());
      }
      return sks;
    }
    if (sk_mode == 1 && sk_plan(a, sks, skl)) {  // skinny bf16 product with pre-transposed weights
      GemmArgs g = a;
      g.ksplit = sks;
      const bool vsk = va && a.lda % 4 == 0;
      const void* kern = vsk ? reinterpret_cast<const void*>(gemm_sk_kernel<true>)
                             : reinterpret_cast<const void*>(gemm_sk_kernel<false>);
      static bool attr_set = false;
      if (!attr_set) {
        TT2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_sk_kernel<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)sk_lds_bytes(SK_KMAX)));
        TT2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_sk_kernel<false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)sk_lds_bytes(SK_KMAX)));
        attr_set = true;
      }
      dim3 grid(cdiv(a.N, SK_BN), 1, sks);
      if (vsk) hipLaunchKernelGGL(gemm_sk_kernel<true>, grid, dim3(256), sk_lds_bytes(skl), s, g, skl);
      else hipLaunchKernelGGL(gemm_sk_kernel<false>, grid, dim3(256), sk_lds_bytes(skl), s, g, skl);
      (void)kern;
      TT2_HIP(hipGetLastError());
      if (sks > 1 && !g.raw) {
        hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(((long)a.M * a.N + 1023) / 1024)), dim3(256), 0, s, g);
        TT2_HIP(hipGetLastError());
      }
      return sks;
    }
    const int wm16 = a.M <= 64 ? 1 : 2;
    GemmArgs g = a;
    g.ksplit = 1;
    const long tiles = (long)cdiv(a.N, 128) * cdiv(a.M, 64 * wm16);
    if (a.kpart) {  // split K until ~kTarget work-groups, >= 4 k tiles (128 k) per split
      static const long kTarget = [] {
        const char* e = std::getenv("TT2_SPLITK16_TARGET");
        return e ? std::max(1L, std::atol(e)) : 512L;
      }();
      int ks = (int)std::min<long>(kTarget / std::max<long>(tiles, 1), cdiv(a.K, X3_BK) / 4);
      ks = std::max(1, std::min(ks, 256));
      while (ks > 1 && (long)ks * a.M * a.N > a.kpart_floats) --ks;
      g.ksplit = ks;
    }
    dim3 grid(cdiv(a.N, 128), cdiv(a.M, 64 * wm16), g.ksplit);
#define TT2_X3(VA_, MODE_, WMB_) hipLaunchKernelGGL((gemm_x3_kernel<VA_, MODE_, WMB_>), grid, dim3(256), 0, s, g)
    if (a.split16 == 1 && a.Bt16) {
#define TT2_X3P(VA_, WMB_) hipLaunchKernelGGL((gemm_x3_kernel<VA_, 1, WMB_, true>), grid, dim3(256), 0, s, g)
      if (wm16 == 2) { if (va) TT2_X3P(true, 2); else TT2_X3P(false, 2); }
      else { if (va) TT2_X3P(true, 1); else TT2_X3P(false, 1); }
#undef TT2_X3P
    } else if (a.split16 == 1) {
      if (wm16 == 2) { if (va) TT2_X3(true, 1, 2); else TT2_X3(false, 1, 2); }
      else { if (va) TT2_X3(true, 1, 1); else TT2_X3(false, 1, 1); }
    } else if (a.Bt16) {
#define TT2_X3B(VA_, WMB_) hipLaunchKernelGGL((gemm_x3_kernel<VA_, 2, WMB_, true>), grid, dim3(256), 0, s, g)
      if (wm16 == 2) { if (va) TT2_X3B(true, 2); else TT2_X3B(false, 2); }
      else { if (va) TT2_X3B(true, 1); else TT2_X3B(false, 1); }
#undef TT2_X3B
    } else {
      if (wm16 == 2) { if (va) TT2_X3(true, 2, 2); else TT2_X3(false, 2, 2); }
      else { if (va) TT2_X3(true, 2, 1); else TT2_X3(false, 2, 1); }
    }
#undef TT2_X3
    TT2_HIP(hipGetLastError());
    if (g.ksplit > 1 && !g.raw) {
      hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(((long)a.M * a.N + 1023) / 1024)), dim3(256), 0, s, g);
      TT2_HIP(hipGetLastError());
    }
    return g.ksplit;
  }
  const bool vb = al16(a.Bw) && (a.ldb % 4 == 0);
  const int wnb = a.N <= 64 ? 1 : 2;
  const long tiles22 = (long)cdiv(a.M, 128) * cdiv(a.N, 64 * wnb);
  const int wmb = tiles22 >= 512 ? 2 : 1;
  GemmArgs g = a;
  g.ksplit = 1;
  if (a.kpart) {  // split K until ~kTarget work-groups, >= 8 k tiles (128 k) per split
    static const long kTarget = [] {
      const char* e = std::getenv("TT2_SPLITK_TARGET");
      return e ? std::max(1L, std::atol(e)) : 512L;
    }();
    const long tiles = (long)cdiv(a.M, 64 * wmb) * cdiv(a.N, 64 * wnb);
    const int nkt = cdiv(a.K, 16);
    int ks = (int)std::min<long>(kTarget / std::max<long>(tiles, 1), nkt / 8);
    ks = std::max(1, std::min(ks, 256));
    while (ks > 1 && (long)ks * a.M * a.N > a.kpart_floats) --ks;
    g.ksplit = ks;
  }
  if (wmb == 2 && wnb == 2) launch<2, 2>(g, va, vb, s);
  else if (wmb == 2) launch<2, 1>(g, va, vb, s);
  else if (wnb == 2) launch<1, 2>(g, va, vb, s);
  else launch<1, 1>(g, va, vb, s);
  if (g.ksplit > 1 && !g.raw) {
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(((long)a.M * a.N + 1023) / 1024)), dim3(256), 0, s, g);
    TT2_HIP(hipGetLastError());
  }
  return g.ksplit;
}

}  // namespace tt2
