// Front end of the configs[4] training step (train_front.h): embedding_lookup (tacotron.py:215-217),
// EncoderRNN bidirectional Zoneout-LSTM (modules.py:283-323, 187-248, training zoneout), the
// ReferenceEncoder's conv2d/BN/ReLU stack and GRU (modules.py:9-64, 499-511) and the GST mlp
// multi-head attention (multihead_attention.py:35-132), forward and backward.  Plain fp32
// elementwise / per-row kernels; the matrix products run as gemm.hip GEMMs from train.hip.
#include "train_front.h"

namespace tt2 {

static inline unsigned fe_blk(long n, int t = 256) { return (unsigned)((n + t - 1) / t); }
__device__ __forceinline__ float fe_sig(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---- embedding --------------------------------------------------------------------------------
__global__ void k_fe_embed(const int* __restrict__ ids, const float* __restrict__ tab, long M, int E,
                           float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * E) return;
  out[i] = tab[(long)ids[i / E] * E + i % E];
}
// d table[s][e] = Σ over positions with id s (deterministic order, one thread per (s, e))
__global__ void k_fe_embed_bwd(const int* __restrict__ ids, const float* __restrict__ dx, long M, int E, int NS,
                               float* __restrict__ dtab) {
  // ids staged 256 at a time in LDS (one coalesced load per chunk instead of a dependent global
  // load per position); every thread still sums its positions in order m = 0..M-1
  __shared__ int sid[256];
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < (long)NS * E;
  const int sym = act ? (int)(i / E) : -1, e = act ? (int)(i % E) : 0;
  float acc = 0.f;
  for (long m0 = 0; m0 < M; m0 += 256) {
    __syncthreads();
    sid[threadIdx.x] = m0 + threadIdx.x < M ? ids[m0 + threadIdx.x] : -2;
    __syncthreads();
    const int n = (int)std::min<long>(256, M - m0);
    for (int jj = 0; jj < n; ++jj)
      if (sid[jj] == sym) acc += dx[(m0 + jj) * E + e];
  }
  if (act) dtab[i] = acc;
}
void fe_embed(const int* ids, const float* table, long M, int E, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_embed, dim3(fe_blk(M * E)), dim3(256), 0, s, ids, table, M, E, out);
}
// Segmented form: blockIdx.y = segment of L positions; part[seg][sym][e] = Σ over the segment's
// positions of that symbol, in position order.  Then a fixed-order sum over the segments.
__global__ void k_fe_embed_bwd_seg(const int* __restrict__ ids, const float* __restrict__ dx, long M, int E, int NS,
                                   long L, float* __restrict__ part) {
  __shared__ int sid[256];
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < (long)NS * E;
  const int sym = act ? (int)(i / E) : -1, e = act ? (int)(i % E) : 0;
  const long m0 = (long)blockIdx.y * L, m1 = std::min<long>(M, m0 + L);
  float acc = 0.f;
  for (long c0 = m0; c0 < m1; c0 += 256) {
    __syncthreads();
    sid[threadIdx.x] = c0 + threadIdx.x < m1 ? ids[c0 + threadIdx.x] : -2;
    __syncthreads();
    const int n = (int)std::min<long>(256, m1 - c0);
    for (int jj = 0; jj < n; ++jj)
      if (sid[jj] == sym) acc += dx[(c0 + jj) * E + e];
  }
  if (act) part[(long)blockIdx.y * NS * E + i] = acc;
}
__global__ void k_fe_embed_bwd_sum(const float* __restrict__ part, int S, long n, float* __restrict__ dtab) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < S; s0 += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s0 + u < S) a[u] += part[(long)(s0 + u) * n + i];
  }
  dtab[i] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}
void fe_embed_bwd(const int* ids, const float* dx, long M, int E, int n_symbols, float* dtable, hipStream_t s,
                  float* scratch, long scratch_floats) {
  const long n = (long)n_symbols * E;
  const int S = (int)std::min<long>(64, (M + 127) / 128);
  if (scratch && S > 1 && (long)S * n <= scratch_floats) {  // positions split over S segments
    const long L = (M + S - 1) / S;
    hipLaunchKernelGGL(k_fe_embed_bwd_seg, dim3(fe_blk(n), S), dim3(256), 0, s, ids, dx, M, E, n_symbols, L, scratch);
    hipLaunchKernelGGL(k_fe_embed_bwd_sum, dim3(fe_blk(n)), dim3(256), 0, s, scratch, S, n, dtable);
    return;
  }
  hipLaunchKernelGGL(k_fe_embed_bwd, dim3(fe_blk(n)), dim3(256), 0, s, ids, dx, M, E, n_symbols, dtable);
}

// ---- BiLSTM -------------------------------------------------------------------------------------
__global__ void k_fe_lstm_cell(FeLstm a) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int B = a.B, U = a.U, T = a.T, t = a.t;
  if (i >= 2L * B * U) return;
  const int dir = (int)(i / ((long)B * U)), b = (int)((i / U) % B), u = (int)(i % U);
  const int len = a.lens[b];
  const long st0 = ((long)dir * (T + 1) + t) * B * U + (long)b * U + u;  // CS/HS at t
  const long st1 = st0 + (long)B * U;                                    // at t+1
  const float cp = a.CS[st0], hp = a.HS[st0];
  if (t >= len) {  // past the row's length: state copied, output stays 0 (TF rnn._rnn_step)
    a.CS[st1] = cp;
    a.HS[st1] = hp;
    return;
  }
  const int pos = dir == 0 ? t : len - 1 - t;
  const float* xp = a.XP + ((long)b * T + pos) * 8 * U + dir * 4 * U;
  const float* gz = a.GZ + ((long)dir * B + b) * 4 * U;
  const float zi = gz[u] + xp[u], zj = gz[U + u] + xp[U + u], zf = gz[2 * U + u] + xp[2 * U + u],
              zo = gz[3 * U + u] + xp[3 * U + u];
  const float si = fe_sig(zi), tj = tanhf(zj), sf = fe_sig(zf + 1.0f), so = fe_sig(zo);
  const float cn = sf * cp + si * tj;
  const float hn = so * tanhf(cn);
  float* ga = a.GA + (((long)dir * T + t) * B + b) * 4 * U;
  ga[u] = si; ga[U + u] = tj; ga[2 * U + u] = sf; ga[3 * U + u] = so;
  a.CN[((long)dir * T + t) * B * U + (long)b * U + u] = cn;
  float mc, mh;
  if (a.zm) {  // training zoneout (modules.py:236-240): keep bits by step
    mc = (float)a.zm[((((long)t * 2 + dir) * 2 + 0) * B + b) * U + u];
    mh = (float)a.zm[((((long)t * 2 + dir) * 2 + 1) * B + b) * U + u];
  } else {
    mc = mh = 1.f - a.zo;
  }
  a.CS[st1] = cp + mc * (cn - cp);
  a.HS[st1] = hp + mh * (hn - hp);
  a.ENC[((long)b * T + pos) * 2 * U + dir * U + u] = hn;
}

__global__ void k_fe_lstm_cell_bwd(FeLstm a) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int B = a.B, U = a.U, T = a.T, t = a.t;
  if (i >= 2L * B * U) return;
  const int dir = (int)(i / ((long)B * U)), b = (int)((i / U) % B), u = (int)(i % U);
  const int len = a.lens[b];
  const long sidx = ((long)dir * B + b) * U + u;
  float* dz = a.DZ + (((long)dir * T + t) * B + b) * 4 * U;
  if (t >= len) {  // copied state: gradients pass through, no gate gradient
    dz[u] = dz[U + u] = dz[2 * U + u] = dz[3 * U + u] = 0.f;
    a.DHP[sidx] = a.DHC[sidx];
    return;
  }
  const int pos = dir == 0 ? t : len - 1 - t;
  const float* ga = a.GA + (((long)dir * T + t) * B + b) * 4 * U;
  const float si = ga[u], tj = ga[U + u], sf = ga[2 * U + u], so = ga[3 * U + u];
  const float cn = a.CN[((long)dir * T + t) * B * U + (long)b * U + u];
  const float cp = a.CS[((long)dir * (T + 1) + t) * B * U + (long)b * U + u];
  float mc, mh;
  if (a.zm) {
    mc = (float)a.zm[((((long)t * 2 + dir) * 2 + 0) * B + b) * U + u];
    mh = (float)a.zm[((((long)t * 2 + dir) * 2 + 1) * B + b) * U + u];
  } else {
    mc = mh = 1.f - a.zo;
  }
  const float dhc = a.DHC[sidx], dcc = a.DCC[sidx];
  const float dout = a.DENC[((long)b * T + pos) * a.ld_denc + dir * U + u];
  const float dhn = dout + mh * dhc;
  const float tc = tanhf(cn);
  const float dcn = mc * dcc + dhn * so * (1.f - tc * tc);
  dz[u] = dcn * tj * si * (1.f - si);
  dz[U + u] = dcn * si * (1.f - tj * tj);
  dz[2 * U + u] = dcn * cp * sf * (1.f - sf);
  dz[3 * U + u] = dhn * tc * so * (1.f - so);
  a.DCC[sidx] = (1.f - mc) * dcc + dcn * sf;
  a.DHP[sidx] = (1.f - mh) * dhc;
}
void fe_lstm_cell(const FeLstm& a, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_lstm_cell, dim3(fe_blk(2L * a.B * a.U)), dim3(256), 0, s, a);
}
void fe_lstm_cell_bwd(const FeLstm& a, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_lstm_cell_bwd, dim3(fe_blk(2L * a.B * a.U)), dim3(256), 0, s, a);
}
__global__ void k_fe_lstm_dxp(const float* __restrict__ DZ, const int* __restrict__ lens, int B, int T, int U,
                              float* __restrict__ dXP) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * T * 8 * U) return;
  const int col = (int)(i % (8 * U));
  const long bp = i / (8 * U);
  const int pos = (int)(bp % T), b = (int)(bp / T);
  const int dir = col / (4 * U), c = col % (4 * U);
  const int len = lens[b];
  float v = 0.f;
  if (pos < len) {
    const int t = dir == 0 ? pos : len - 1 - pos;
    v = DZ[(((long)dir * T + t) * B + b) * 4 * U + c];
  }
  dXP[i] = v;
}
void fe_lstm_dxp(const float* DZ, const int* lens, int B, int T, int U, float* dXP, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_lstm_dxp, dim3(fe_blk((long)B * T * 8 * U)), dim3(256), 0, s, DZ, lens, B, T, U, dXP);
}

// ---- reference encoder ---------------------------------------------------------------------------
__global__ void k_fe_bn_relu_fwd(const float* __restrict__ a, long M, int C, const float* __restrict__ mean,
                                 const float* __restrict__ var, const float* __restrict__ gamma,
                                 const float* __restrict__ beta, float eps, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  y[i] = fmaxf(gamma[c] * (a[i] - mean[c]) * rsqrtf(var[c] + eps) + beta[c], 0.f);
}
void fe_bn_relu_fwd(const float* a, long M, int C, const float* mean, const float* var, const float* gamma,
                    const float* beta, float eps, float* y, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_bn_relu_fwd, dim3(fe_blk(M * C)), dim3(256), 0, s, a, M, C, mean, var, gamma, beta, eps, y);
}
__global__ void k_fe_relu_mask(const float* __restrict__ dy, const float* __restrict__ y, long n,
                               float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = y[i] > 0.f ? dy[i] : 0.f;
}
void fe_relu_mask(const float* dy, const float* y, long n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_relu_mask, dim3(fe_blk(n)), dim3(256), 0, s, dy, y, n, out);
}
// out[((i*3 + j)*C + c) * ldo + m] = x(n, st ho + i - pt, st wo + j - pl, c), m = (n*Ho + ho)*Wo + wo.
// Grid (M / 256, 9 C): the column k = (i*3 + j)*C + c is the block's y (uniform), m the thread's x, so
// the stores of a wave are one contiguous run and the index arithmetic is 32-bit (the 1-D form's
// 64-bit i / M, i % M per element bound it at 0.5 TB/s)
__global__ __launch_bounds__(256) void k_fe_im2col2d_t(const float* __restrict__ x, int N, int H, int W, int C, int Ho,
                                                       int Wo, int pt, int pl, float* __restrict__ out, long ldo, int st) {
  const int M = N * Ho * Wo;
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const int k = blockIdx.y, c = k % C, ij = k / C, ii = ij / 3, jj = ij - 3 * ii;
  const int wo = m % Wo, r = m / Wo, ho = r % Ho, n = r / Ho;
  const int h = st * ho + ii - pt, w = st * wo + jj - pl;
  out[(long)k * ldo + m] = (h >= 0 && h < H && w >= 0 && w < W) ? x[((long)(n * H + h) * W + w) * C + c] : 0.f;
}
void fe_im2col2d_t(const float* x, int N, int H, int W, int C, int Ho, int Wo, int pt, int pl, float* out, long ldo,
                   hipStream_t s, int st) {
  const long M = (long)N * Ho * Wo;
  TT2_CHECK(M < (1L << 31) && 9L * C <= 65535, TT2_ERR_SHAPE_MISMATCH, "im2col2d: shape exceeds the 32-bit grid");
  hipLaunchKernelGGL(k_fe_im2col2d_t, dim3((unsigned)((M + 255) / 256), 9 * C), dim3(256), 0, s, x, N, H, W, C, Ho, Wo,
                     pt, pl, out, ldo, st);
}
// dx(n, h, w, c) = Σ_{i,j} dcols[(n, ho, wo)][(i*3+j)*C + c] over the outputs whose taps read it
// (32-bit index arithmetic; stride 1 / 2 as a uniform branch)
__global__ __launch_bounds__(256) void k_fe_col2im2d(const float* __restrict__ dcols, int N, int H, int W, int C, int Ho,
                                                     int Wo, int pt, int pl, float* __restrict__ dx, int st) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * H * W * C) return;
  const int c = i % C, r0 = i / C, w = r0 % W, r1 = r0 / W, h = r1 % H, n = r1 / H;
  float acc = 0.f;
#pragma unroll
  for (int ii = 0; ii < 3; ++ii) {
    const int hh = h + pt - ii;
    const int ho = st == 1 ? hh : hh >> 1;
    if (hh < 0 || (st != 1 && (hh & 1)) || ho >= Ho) continue;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const int ww = w + pl - jj;
      const int wo = st == 1 ? ww : ww >> 1;
      if (ww < 0 || (st != 1 && (ww & 1)) || wo >= Wo) continue;
      const long m = (long)(n * Ho + ho) * Wo + wo;
      acc += dcols[m * 9 * C + (ii * 3 + jj) * C + c];
    }
  }
  dx[i] = acc;
}
void fe_col2im2d(const float* dcols, int N, int H, int W, int C, int Ho, int Wo, int pt, int pl, float* dx,
                 hipStream_t s, int st) {
  const long n = (long)N * H * W * C;
  TT2_CHECK(n < (1L << 31) && (st == 1 || st == 2), TT2_ERR_SHAPE_MISMATCH, "col2im2d: shape / stride unsupported");
  hipLaunchKernelGGL(k_fe_col2im2d, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dcols, N, H, W, C, Ho, Wo, pt,
                     pl, dx, st);
}

// ---- direct conv2d backward (no materialised im2col) ------------------------------------------------
// d kernel of a 3x3 conv2d (stride st, 'same' pads pt / pl) over NHWC x [N][H][W][C] and dz [M][F]
// (M = N·Ho·Wo): dW[(tap·C + c)·F + f] = Σ_m x(patch of m)[tap][c] · dz[m][f], fp32 FMA.  Work-group
// = a run of output positions staged PC at a time in LDS ([PC][9C] patches, [PC][F] dz rows);
// thread tile = channel c × 4 columns f over the 9 taps (R tiles when C·F/4 > 256; G position
// groups when it is < 256); one partial row [9CF] per (work-group, group), summed by the caller.
template <int R>
__global__ __launch_bounds__(256) void k_fe_conv2d_dw(const float* __restrict__ x, const float* __restrict__ dz, int N,
                                                      int H, int W, int C, int Ho, int Wo, int F, int pt, int pl,
                                                      int st, int ppb, int PC, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int K9 = 9 * C, T = C * F / 4, Tt = T < 256 ? T : 256, G = 256 / Tt;
  const int tid = threadIdx.x, pg = tid / Tt, q0 = tid % Tt;
  float* const xs = fsm;             // [PC][9C]
  float* const ds = fsm + PC * K9;   // [PC][F]
  const int M = N * Ho * Wo;
  const int m0 = blockIdx.x * ppb, m1 = min(M, m0 + ppb);
  float acc[R][9][4];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[r][k][j] = 0.f;
  for (int p0 = m0; p0 < m1; p0 += PC) {
    const int np = min(PC, m1 - p0);
    for (int e = tid; e < np * C; e += 256) {  // one position decomposition per (p, c), the 9 taps inside
      const int p = e / C, c = e - p * C;
      const int m = p0 + p, wo = m % Wo, rr = m / Wo, ho = rr % Ho, n = rr / Ho;
      const int hb = st * ho - pt, wb = st * wo - pl;
      const float* xb = x + (long)n * H * W * C + c;
      float* xd = xs + p * K9 + c;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int h = hb + ky;
        const bool hv = h >= 0 && h < H;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int w = wb + kx;
          xd[(ky * 3 + kx) * C] = (hv && w >= 0 && w < W) ? xb[((long)h * W + w) * C] : 0.f;
        }
      }
    }
    for (int e = tid; e < np * F / 4; e += 256)
      reinterpret_cast<float4*>(ds)[e] = reinterpret_cast<const float4*>(dz + (long)p0 * F)[e];
    __syncthreads();
    for (int p = pg; p < np; p += G) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int q = q0 + 256 * r, c = q / (F / 4), ng = q % (F / 4);
        const float4 d4 = reinterpret_cast<const float4*>(ds + p * F)[ng];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const float xv = xs[p * K9 + k * C + c];
          acc[r][k][0] += xv * d4.x;
          acc[r][k][1] += xv * d4.y;
          acc[r][k][2] += xv * d4.z;
          acc[r][k][3] += xv * d4.w;
        }
      }
    }
    __syncthreads();
  }
  float* const out = part + ((long)blockIdx.x * G + pg) * K9 * F;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = q0 + 256 * r, c = q / (F / 4), ng = q % (F / 4);
#pragma unroll
    for (int k = 0; k < 9; ++k)
      reinterpret_cast<float4*>(out + (k * C + c) * F)[ng] = make_float4(acc[r][k][0], acc[r][k][1], acc[r][k][2], acc[r][k][3]);
  }
}
bool fe_conv2d_dw_ok(int C, int F) {
  const int T = C * F / 4;
  return F % 4 == 0 && T >= 1 && (T <= 256 ? 256 % T == 0 : (T % 256 == 0 && T / 256 <= 4)) &&
         9 * C + F <= 24576 / 8;
}
int fe_conv2d_dw(const float* x, const float* dz, int N, int H, int W, int C, int Ho, int Wo, int F, int pt, int pl,
                 int st, float* part, long part_floats, hipStream_t s) {
  TT2_CHECK(fe_conv2d_dw_ok(C, F), TT2_ERR_SHAPE_MISMATCH, "conv2d_dw: unsupported channel counts");
  const long M = (long)N * Ho * Wo;
  TT2_CHECK(M < (1L << 31) && (long)N * H * W * C < (1L << 31), TT2_ERR_SHAPE_MISMATCH, "conv2d_dw: shape exceeds 32 bits");
  const int K9 = 9 * C, T = C * F / 4, G = T < 256 ? 256 / T : 1, R = T > 256 ? T / 256 : 1;
  // chunks of PC positions (<= 40 KB of LDS: several work-groups per CU), ~1024 work-groups
  const int PC = std::max(8, std::min(128, 10240 / (K9 + F)) / 8 * 8);
  const long rows_cap = part_floats / ((long)K9 * F * G);
  long nblk = std::min<long>({1024L, (M + PC - 1) / PC, rows_cap});
  TT2_CHECK(nblk >= 1, TT2_ERR_SHAPE_MISMATCH, "conv2d_dw: partial buffer too small");
  const int ppb = (int)(((M + nblk - 1) / nblk + PC - 1) / PC * PC);
  nblk = (M + ppb - 1) / ppb;
  const size_t lds = sizeof(float) * (size_t)PC * (K9 + F);
  static bool attr = false;
  if (!attr) {
    for (const void* k : {reinterpret_cast<const void*>(k_fe_conv2d_dw<1>), reinterpret_cast<const void*>(k_fe_conv2d_dw<2>),
                          reinterpret_cast<const void*>(k_fe_conv2d_dw<4>)})
      TT2_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    attr = true;
  }
  const dim3 grid((unsigned)nblk);
  if (R == 1) hipLaunchKernelGGL(k_fe_conv2d_dw<1>, grid, dim3(256), lds, s, x, dz, N, H, W, C, Ho, Wo, F, pt, pl, st, ppb, PC, part);
  else if (R == 2) hipLaunchKernelGGL(k_fe_conv2d_dw<2>, grid, dim3(256), lds, s, x, dz, N, H, W, C, Ho, Wo, F, pt, pl, st, ppb, PC, part);
  else hipLaunchKernelGGL(k_fe_conv2d_dw<4>, grid, dim3(256), lds, s, x, dz, N, H, W, C, Ho, Wo, F, pt, pl, st, ppb, PC, part);
  TT2_HIP(hipGetLastError());
  return (int)(nblk * G);  // partial rows of [9CF]
}

// forward of a 3x3 conv2d with few input channels (the refnets' first layer reads the 1-channel mel):
// out[m][f] = bias[f] + Σ_{tap, c} x(patch of m)[tap][c] · Wk[tap][c][f] (+ ReLU), fp32 products and
// sums.  Thread = (output position, 4 columns); the kernel and bias staged in LDS.  bf: operands
// rounded to bf16 first, as the bf16 step's GEMM form rounds them.  The implicit-GEMM form padded K = 9
// to its 32-deep tile and used 32 of its 128 columns (184 us per refnet at configs[4])
__global__ __launch_bounds__(256) void k_fe_conv2d_fwd_small(const float* __restrict__ x, const float* __restrict__ Wk,
                                                             const float* __restrict__ bias, int N, int H, int W, int C,
                                                             int Ho, int Wo, int F, int pt, int pl, int st, int relu,
                                                             int bf, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  for (int e = threadIdx.x; e < 9 * C * F; e += 256) fsm[e] = bf ? (float)(__bf16)Wk[e] : Wk[e];
  for (int e = threadIdx.x; e < F; e += 256) fsm[9 * C * F + e] = bias[e];
  __syncthreads();
  const int FQ = F / 4;
  const int total = N * Ho * Wo * FQ;  // < 2^31 (host check): 32-bit index arithmetic
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int fq = i % FQ, m = i / FQ;
    const int wo = m % Wo, r = m / Wo, ho = r % Ho, n = r / Ho;
    f32x4 acc = *reinterpret_cast<const f32x4*>(fsm + 9 * C * F + 4 * fq);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int h = st * ho + ky - pt;
      if (h < 0 || h >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int w = st * wo + kx - pl;
        if (w < 0 || w >= W) continue;
        const float* xp = x + ((long)(n * H + h) * W + w) * C;
        const float* wp = fsm + (ky * 3 + kx) * C * F + 4 * fq;
        for (int c = 0; c < C; ++c) acc += (bf ? (float)(__bf16)xp[c] : xp[c]) * *reinterpret_cast<const f32x4*>(wp + c * F);
      }
    }
    if (relu)
      for (int u = 0; u < 4; ++u) acc[u] = fmaxf(acc[u], 0.f);
    *reinterpret_cast<f32x4*>(out + (long)m * F + 4 * fq) = acc;
  }
}
bool fe_conv2d_fwd_small_ok(int C, int F) { return C >= 1 && C <= 4 && F % 4 == 0 && 9 * C * F + F <= 8192; }
void fe_conv2d_fwd_small(const float* x, const float* Wk, const float* bias, int N, int H, int W, int C, int Ho, int Wo,
                         int F, int pt, int pl, int st, bool relu, float* out, hipStream_t s, bool bf16) {
  TT2_CHECK(fe_conv2d_fwd_small_ok(C, F), TT2_ERR_SHAPE_MISMATCH, "conv2d_fwd_small: unsupported channel counts");
  const long total = (long)N * Ho * Wo * (F / 4);
  TT2_CHECK(total < (1L << 31) && (long)N * H * W * C < (1L << 31), TT2_ERR_SHAPE_MISMATCH,
            "conv2d_fwd_small: shape exceeds 32 bits");
  const unsigned nb = (unsigned)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(k_fe_conv2d_fwd_small, dim3(nb), dim3(256), sizeof(float) * (size_t)(9 * C * F + F), s, x, Wk, bias,
                     N, H, W, C, Ho, Wo, F, pt, pl, st, relu ? 1 : 0, bf16 ? 1 : 0, out);
  TT2_HIP(hipGetLastError());
}

// d input of the same conv2d as a gather: dx[n][h][w][c] = Σ_{taps reading (h, w)} Σ_f dz[n][ho][wo][f] ·
// Wk[tap][c][f] (Wk the HWIO kernel [3][3][C][F]).  Work-group = DXR consecutive rows h of one image:
// the kernel (as [tap][f][C]) and the dz rows those rows read are staged in LDS once; thread item =
// 4 channels × DXW positions w0 + st·k of one row (equal w parity: one tap pattern), so each weight
// float4 feeds 4·DXW FMAs and the dz quads are LDS broadcasts across the channel groups.
constexpr int DXW = 4, DXR = 16;
template <int st>
__global__ __launch_bounds__(256) void k_fe_conv2d_dx(const float* __restrict__ dz, const float* __restrict__ Wk, int N,
                                                      int H, int W, int C, int Ho, int Wo, int F, int pt, int pl,
                                                      float* __restrict__ dx) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int bpi = (H + DXR - 1) / DXR, n = blockIdx.x / bpi, h0 = (blockIdx.x % bpi) * DXR, h1 = min(H, h0 + DXR);
  // dz rows [r0, r1) feed rows [h0, h1): ho = (h + pt - ky) / st
  const int r0 = max(0, (h0 + pt - 2 + st - 1) / st), r1 = min(Ho, (h1 - 1 + pt) / st + 1);
  const int Fp = F + 4;                 // padded dz position stride: lanes of consecutive positions
                                        // hit different LDS banks
  float* const wt = fsm;                // [9][F][C]
  float* const ds = fsm + 9 * C * F;    // [r1 - r0][Wo][Fp], then one zero position (taps off the map)
  for (int e = threadIdx.x; e < 9 * C * F; e += 256) {  // Wk[(tap·C + c)·F + f] -> [(tap·F + f)·C + c]
    const int f = e % F, tc = e / F, c = tc % C, tap = tc / C;
    wt[(tap * F + f) * C + c] = Wk[e];
  }
  const int F4 = F / 4, nd = max(0, r1 - r0) * Wo * F4;
  const float4* dsrc = reinterpret_cast<const float4*>(dz + ((long)n * Ho + r0) * Wo * F);
  for (int e = threadIdx.x; e < nd; e += 256) {
    const int pos = e / F4, f4 = e - pos * F4;
    *reinterpret_cast<float4*>(ds + pos * Fp + 4 * f4) = dsrc[e];
  }
  float* const dzero = ds + max(0, r1 - r0) * Wo * Fp;
  for (int e = threadIdx.x; e < F; e += 256) dzero[e] = 0.f;
  __syncthreads();
  // wave item = (row h, w parity): its lanes are (channel group, w block), so the tap pattern is
  // wave-uniform (no divergence on the stride-2 parity tests)
  const int CG = C / 4, WB = (W + st * DXW - 1) / (st * DXW);
  const int lane = threadIdx.x & 63, cg = lane % CG;
  const bool act = lane / CG < WB;            // lanes past the row's w blocks compute block 0 and store nothing
  const int wb = act ? lane / CG : 0;         // (no divergent region around the tap branches)
  const int nwi = (h1 - h0) * st;
  for (int wi = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); wi < nwi; wi += 4) {  // wave-uniform (SGPR)
    const int par = wi % st, h = h0 + wi / st;
    const int w0 = par + st * wb;  // position k: w0 + st·WB·k (consecutive lanes, consecutive positions)
    float acc[DXW][4] = {};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int hh = h + pt - ky;
      if (hh < 0 || hh % st) continue;
      const int ho = hh / st;
      if (ho >= Ho) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ww0 = w0 + pl - kx;  // + st·WB·k for position k
        if ((((par + pl - kx) % st) + st) % st) continue;  // = ww0's parity, written wave-uniform
        const float* wp = wt + (ky * 3 + kx) * F * C + 4 * cg;
        const float* dr[DXW];  // positions off the map read the zero row: no branches in the f loop
#pragma unroll
        for (int k = 0; k < DXW; ++k) {
          const int ww = ww0 + st * WB * k, wo = ww >= 0 ? ww / st : 0;
          dr[k] = (ww >= 0 && wo < Wo) ? ds + ((ho - r0) * Wo + wo) * Fp : dzero;
        }
        for (int f = 0; f < F; f += 4) {
          float4 dv[DXW];
#pragma unroll
          for (int k = 0; k < DXW; ++k) dv[k] = *reinterpret_cast<const float4*>(dr[k] + f);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float4 w4 = *reinterpret_cast<const float4*>(wp + (f + j) * C);
#pragma unroll
            for (int k = 0; k < DXW; ++k) {
              const float d = j == 0 ? dv[k].x : j == 1 ? dv[k].y : j == 2 ? dv[k].z : dv[k].w;
              acc[k][0] += d * w4.x;
              acc[k][1] += d * w4.y;
              acc[k][2] += d * w4.z;
              acc[k][3] += d * w4.w;
            }
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < DXW; ++k) {
      const int w = w0 + st * WB * k;
      if (act && w < W)
        *reinterpret_cast<float4*>(dx + ((long)(n * H + h) * W + w) * C + 4 * cg) =
            make_float4(acc[k][0], acc[k][1], acc[k][2], acc[k][3]);
    }
  }
}
static long fe_dx_lds_floats(int C, int Ho, int Wo, int F, int st) {
  const int rows = std::min(Ho, (DXR + 2) / st + 2);
  return 9L * C * F + (long)rows * Wo * (F + 4) + F;
}
// F <= 32: at refnet layer 2 (C 32, F 64: 102 KB of LDS, one work-group per CU) it measured 440 us against
// the GEMM + col2im form's ~150; at layer 1 (C = F = 32) 266 against 421
bool fe_conv2d_dx_ok(int C, int W, int Ho, int Wo, int F, int st) {  // LDS budget; one wave covers a row
  return C % 4 == 0 && F % 4 == 0 && F <= 32 && (st == 1 || st == 2) && fe_dx_lds_floats(C, Ho, Wo, F, st) * 4 <= 120 * 1024 &&
         (C / 4) * ((W + st * DXW - 1) / (st * DXW)) <= 64;
}
void fe_conv2d_dx(const float* dz, const float* Wk, int N, int H, int W, int C, int Ho, int Wo, int F, int pt, int pl,
                  int st, float* dx, hipStream_t s) {
  TT2_CHECK(fe_conv2d_dx_ok(C, W, Ho, Wo, F, st), TT2_ERR_SHAPE_MISMATCH, "conv2d_dx: unsupported shape");
  TT2_CHECK((long)N * Ho * Wo * F < (1L << 31) && (long)N * H * W * C < (1L << 31), TT2_ERR_SHAPE_MISMATCH,
            "conv2d_dx: shape exceeds 32 bits");
  const long lds = sizeof(float) * fe_dx_lds_floats(C, Ho, Wo, F, st);
  static bool attr = false;
  if (!attr) {
    for (const void* k : {reinterpret_cast<const void*>(k_fe_conv2d_dx<1>), reinterpret_cast<const void*>(k_fe_conv2d_dx<2>)})
      TT2_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
    attr = true;
  }
  const unsigned nb = (unsigned)((long)N * ((H + DXR - 1) / DXR));
  if (st == 1) hipLaunchKernelGGL(k_fe_conv2d_dx<1>, dim3(nb), dim3(256), (size_t)lds, s, dz, Wk, N, H, W, C, Ho, Wo, F, pt, pl, dx);
  else hipLaunchKernelGGL(k_fe_conv2d_dx<2>, dim3(nb), dim3(256), (size_t)lds, s, dz, Wk, N, H, W, C, Ho, Wo, F, pt, pl, dx);
  TT2_HIP(hipGetLastError());
}

// ---- ReferenceEncoderAdaIn (modules.py:89-98) ------------------------------------------------------
// per (row, channel) moments over the HW positions of NHWC x [N][HW][C] (tf.nn.moments axes [1, 2]:
// biased variance): mv[(n*C + c)*2 + {0: mean, 1: var}].  Work-group (n, 64-channel block): 4 row
// groups of 64 lanes, two passes (mean, then Σ (x - mean)²)
__global__ __launch_bounds__(256) void k_fe_ad_moments(const float* __restrict__ x, int HW, int C,
                                                       float* __restrict__ mv) {
  __shared__ float red[4][64];
  const int n = blockIdx.x, c = blockIdx.y * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const bool ok = c < C;
  const float* xr = x + (long)n * HW * C;
  float s = 0.f;
  if (ok)
    for (int p = g; p < HW; p += 4) s += xr[(long)p * C + c];
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  const float mean = ((red[0][threadIdx.x & 63] + red[1][threadIdx.x & 63]) +
                      (red[2][threadIdx.x & 63] + red[3][threadIdx.x & 63])) / (float)HW;
  __syncthreads();
  float q = 0.f;
  if (ok)
    for (int p = g; p < HW; p += 4) {
      const float d = xr[(long)p * C + c] - mean;
      q += d * d;
    }
  red[g][threadIdx.x & 63] = q;
  __syncthreads();
  if (ok && g == 0) {
    const int l = threadIdx.x;
    mv[((long)n * C + c) * 2] = mean;
    mv[((long)n * C + c) * 2 + 1] = ((red[0][l] + red[1][l]) + (red[2][l] + red[3][l])) / (float)HW;
  }
}
void fe_ad_moments(const float* x, int N, int HW, int C, float* mv, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_ad_moments, dim3(N, (C + 63) / 64), dim3(256), 0, s, x, HW, C, mv);
}
// y = 0.9 xs + 0.1 tf.nn.batch_normalization(xs, m_s, v_s, offset = m_e, scale = v_e, 1e-9)
//   = 0.9 xs + 0.1 (xs inv + (m_e - m_s inv)), inv = v_e / sqrt(v_s + 1e-9)
__global__ void k_fe_ad_mix(const float* __restrict__ xs, long n, int HW, int C, const float* __restrict__ mv_s,
                            const float* __restrict__ mv_e, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long r = i / ((long)HW * C);
  const int c = (int)(i % C);
  const long q = (r * C + c) * 2;
  const float inv = mv_e[q + 1] / sqrtf(mv_s[q + 1] + 1e-9f);
  y[i] = xs[i] * 0.9f + (xs[i] * inv + (mv_e[q] - mv_s[q] * inv)) * 0.1f;
}
void fe_ad_mix(const float* xs, int N, int HW, int C, const float* mv_s, const float* mv_e, float* y, hipStream_t s) {
  const long n = (long)N * HW * C;
  hipLaunchKernelGGL(k_fe_ad_mix, dim3(fe_blk(n)), dim3(256), 0, s, xs, n, HW, C, mv_s, mv_e, y);
}
// backward of the mix, g = 0.1 dy, x̂ = (xs - m_s) / sqrt(v_s + 1e-9), per (row, channel) over N = HW:
//   S1 = Σ g, S2 = Σ g x̂
//   d xs = 0.9 dy + inv (g - S1 / N - x̂ S2 / N)          (m_s, v_s are functions of xs)
//   d xe = S1 / N + S2 · 2 (xe - m_e) / N                  (offset m_e, scale v_e: d m_e = S1, d v_e = S2)
__global__ __launch_bounds__(256) void k_fe_ad_mix_sums(const float* __restrict__ dy, const float* __restrict__ xs,
                                                        int HW, int C, const float* __restrict__ mv_s,
                                                        float* __restrict__ S) {
  __shared__ float r1[4][64], r2[4][64];
  const int n = blockIdx.x, c = blockIdx.y * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6, l = threadIdx.x & 63;
  const bool ok = c < C;
  float s1 = 0.f, s2 = 0.f;
  if (ok) {
    const long q = ((long)n * C + c) * 2;
    const float m = mv_s[q], rs = 1.0f / sqrtf(mv_s[q + 1] + 1e-9f);
    const long base = (long)n * HW * C + c;
    for (int p = g; p < HW; p += 4) {
      const float gg = 0.1f * dy[base + (long)p * C];
      s1 += gg;
      s2 += gg * ((xs[base + (long)p * C] - m) * rs);
    }
  }
  r1[g][l] = s1;
  r2[g][l] = s2;
  __syncthreads();
  if (ok && g == 0) {
    S[((long)n * C + c) * 2] = (r1[0][l] + r1[1][l]) + (r1[2][l] + r1[3][l]);
    S[((long)n * C + c) * 2 + 1] = (r2[0][l] + r2[1][l]) + (r2[2][l] + r2[3][l]);
  }
}
__global__ void k_fe_ad_mix_bwd(const float* __restrict__ dy, const float* __restrict__ xs,
                                const float* __restrict__ xe, long n, int HW, int C, const float* __restrict__ mv_s,
                                const float* __restrict__ mv_e, const float* __restrict__ S, float* __restrict__ dxs,
                                float* __restrict__ dxe) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long r = i / ((long)HW * C);
  const int c = (int)(i % C);
  const long q = (r * C + c) * 2;
  const float rs = 1.0f / sqrtf(mv_s[q + 1] + 1e-9f), inv = mv_e[q + 1] * rs, N = (float)HW;
  const float xh = (xs[i] - mv_s[q]) * rs, g = 0.1f * dy[i];
  dxs[i] = 0.9f * dy[i] + inv * (g - S[q] / N - xh * S[q + 1] / N);
  dxe[i] = S[q] / N + S[q + 1] * 2.f * (xe[i] - mv_e[q]) / N;
}
void fe_ad_mix_bwd(const float* dy, const float* xs, const float* xe, int N, int HW, int C, const float* mv_s,
                   const float* mv_e, float* S, float* dxs, float* dxe, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_ad_mix_sums, dim3(N, (C + 63) / 64), dim3(256), 0, s, dy, xs, HW, C, mv_s, S);
  const long n = (long)N * HW * C;
  hipLaunchKernelGGL(k_fe_ad_mix_bwd, dim3(fe_blk(n)), dim3(256), 0, s, dy, xs, xe, n, HW, C, mv_s, mv_e, S, dxs, dxe);
}

// GRU step t, part a: [r, u] = σ(XG_g + h·Wg_h); RH = r·h
__global__ void k_fe_gru_a(const float* __restrict__ XG, const float* __restrict__ GG, const float* __restrict__ HG,
                           int N, int T2, int D, int t, float* __restrict__ R, float* __restrict__ Uu,
                           float* __restrict__ RH) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const int n = i / D, d = i % D;
  const float* xg = XG + ((long)n * T2 + t) * 3 * D;
  const float r = fe_sig(xg[d] + GG[(long)n * 2 * D + d]);
  const float u = fe_sig(xg[D + d] + GG[(long)n * 2 * D + D + d]);
  const long o = ((long)t * N + n) * D + d;
  R[o] = r;
  Uu[o] = u;
  RH[o] = r * HG[o];  // HG[t] = h(t), step-major [T2+1][N][D]
}
// part b: c = tanh(XG_c + (r·h)·Wc_h); h(t+1) = u·h + (1 - u)·c
__global__ void k_fe_gru_b(const float* __restrict__ XG, const float* __restrict__ GC, const float* __restrict__ Uu,
                           int N, int T2, int D, int t, float* __restrict__ CC, float* __restrict__ HG) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const int n = i / D, d = i % D;
  const float c = tanhf(XG[((long)n * T2 + t) * 3 * D + 2 * D + d] + GC[(long)n * D + d]);
  const long o = ((long)t * N + n) * D + d;
  const float u = Uu[o];
  CC[o] = c;
  HG[o + (long)N * D] = u * HG[o] + (1.f - u) * c;
}
// ---- the whole GRU recurrence of one reference encoder in one work-group -----------------------------
// (modules.py:59, TF1 GRUCell; the per-step form above is 4 launches + split-K combines per step).  1024
// threads; the recurrent weights live in registers as v_mfma_f32_16x16x4f32 B fragments (exact fp32
// products), the step's A operands (h, r·h forward; d candidate, d gates backward) in LDS with k
// permuted so a lane's four consecutive k-steps are one 16-byte read.  Rows >= N are never consumed
// (MFMA rows are independent).  Same outputs as the per-step kernels: R, U, RH, CC, HG[t+1] forward;
// DCP, DGP and the running d h backward.
template <int KS4>
__device__ __forceinline__ void gru_mm(f32x4 (&acc)[4], const float* AL, int ld, int K4, int s0, const float (&bf)[KS4],
                                       int lane) {
  const int r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int c = 0; c < KS4; c += 4) {
    f32x4 a[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) a[mt] = *reinterpret_cast<const f32x4*>(AL + (16 * mt + r) * ld + g * K4 + s0 + c);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][j], bf[c + j], acc[mt], 0, 0, 0);
    asm volatile("" ::: "memory");  // keep the next group's LDS reads below: 16 operand registers live, not 128
  }
}
// C fragment (rows 16 mt + 4 (lane >> 4) + i, column col0 + (lane & 15)) -> P[row][col] (row stride ldp)
__device__ __forceinline__ void gru_put(const f32x4 (&acc)[4], float* P, int ldp, int col0, int lane) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) P[(16 * mt + 4 * (lane >> 4) + i) * ldp + col0 + (lane & 15)] = acc[mt][i];
}
// k -> its slot in a permuted A row of K columns (k = 4 s + g at g·K/4 + s)
__device__ __forceinline__ int gru_perm(int k, int K) { return (k & 3) * (K >> 2) + (k >> 2); }

// LDS-only work-group barrier: every barrier in the recurrences orders LDS data only, while a
// __syncthreads() would also wait for the step's global stores (R, U, ... read only after the launch)
__device__ __forceinline__ void gru_lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
constexpr int GRU_NT = 512, GRU_NW = GRU_NT / 64;  // 8 waves: 256 registers per lane for the weight fragments
template <int RD>
__global__ __launch_bounds__(GRU_NT) void k_fe_gru_fwd_seq(const float* __restrict__ XG, const float* __restrict__ Wgh,
                                                          const float* __restrict__ Wch, int N, int T2,
                                                          float* __restrict__ R, float* __restrict__ Uo,
                                                          float* __restrict__ RHo, float* __restrict__ CC,
                                                          float* __restrict__ HG) {
  constexpr int KS = RD / 4, LD = RD + 4, NTG = 2 * RD / 16, NTC = RD / 16, EPT = 64 * RD / GRU_NT;
  constexpr int UG = (NTG + GRU_NW - 1) / GRU_NW, UC = (2 * NTC + GRU_NW - 1) / GRU_NW;  // units per wave
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* const hL = fsm;            // h(t) rows, permuted k
  float* const rL = hL + 64 * LD;   // r·h rows
  float* const P = rL + 64 * LD;    // GG [64][2RD], then the GC halves [2][64][RD]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g4 = lane >> 4, cl = lane & 15;
  float bg[UG][KS], bc[UC][KS / 2];  // GG unit j: column tile w + 8 j; GC unit j: u = w + 8 j -> tile u % NTC, k half u / NTC
#pragma unroll
  for (int j = 0; j < UG; ++j)
#pragma unroll
    for (int s = 0; s < KS; ++s) bg[j][s] = w + GRU_NW * j < NTG ? Wgh[(4 * s + g4) * 2 * RD + 16 * (w + GRU_NW * j) + cl] : 0.f;
#pragma unroll
  for (int j = 0; j < UC; ++j) {
    const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
#pragma unroll
    for (int s = 0; s < KS / 2; ++s) bc[j][s] = u < 2 * NTC ? Wch[(4 * (kh * KS / 2 + s) + g4) * RD + 16 * ct + cl] : 0.f;
  }
  for (int e = tid; e < 2 * 64 * LD; e += GRU_NT) fsm[e] = 0.f;  // h(0) = 0
  float uu[EPT];
  __syncthreads();
  for (int t = 0; t < T2; ++t) {
    int tq = tid;
    asm volatile("" : "+v"(tq));  // per-step element addresses recomputed, not hoisted (and spilled) across the loop
#pragma unroll
    for (int j = 0; j < UG; ++j)
      if (w + GRU_NW * j < NTG) {  // GG = h·Wg_h, column tile w + 8 j
        f32x4 acc[4] = {};
        gru_mm<KS>(acc, hL, LD, KS, 0, bg[j], lane);
        gru_put(acc, P, 2 * RD, 16 * (w + GRU_NW * j), lane);
      }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {  // [r, u] = σ(XG_g + GG); RH = r·h
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const float* xg = XG + ((long)n * T2 + t) * 3 * RD;
        const float r = fe_sig(xg[d] + P[n * 2 * RD + d]);
        const float u = fe_sig(xg[RD + d] + P[n * 2 * RD + RD + d]);
        const long o = ((long)t * N + n) * RD + d;
        const float rh = r * hL[n * LD + gru_perm(d, RD)];
        R[o] = r;
        Uo[o] = u;
        RHo[o] = rh;
        rL[n * LD + gru_perm(d, RD)] = rh;
        uu[i] = u;
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int j = 0; j < UC; ++j) {
      const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
      if (u < 2 * NTC) {  // GC = (r·h)·Wc_h, column tile ct, k half kh
        f32x4 acc[4] = {};
        gru_mm<KS / 2>(acc, rL, LD, KS, kh * KS / 2, bc[j], lane);
        gru_put(acc, P + kh * 64 * RD, RD, 16 * ct, lane);
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {  // c = tanh(XG_c + GC); h(t+1) = u·h + (1 - u)·c
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const float c = tanhf(XG[((long)n * T2 + t) * 3 * RD + 2 * RD + d] + (P[n * RD + d] + P[64 * RD + n * RD + d]));
        const long o = ((long)t * N + n) * RD + d;
        const int hi = n * LD + gru_perm(d, RD);
        const float hn = uu[i] * hL[hi] + (1.f - uu[i]) * c;
        CC[o] = c;
        HG[o + (long)N * RD] = hn;
        hL[hi] = hn;
      }
    }
    gru_lds_bar();
  }
}

template <int RD>
__global__ __launch_bounds__(GRU_NT) void k_fe_gru_bwd_seq(const float* __restrict__ Wgh, const float* __restrict__ Wch,
                                                          const float* __restrict__ R, const float* __restrict__ Uu,
                                                          const float* __restrict__ CC, const float* __restrict__ HG,
                                                          int N, int T2, float* __restrict__ dH, float* __restrict__ DCP,
                                                          float* __restrict__ DGP) {
  constexpr int KS = RD / 4, L1 = RD + 4, L2 = 2 * RD + 4, NTC = RD / 16, EPT = 64 * RD / GRU_NT;
  constexpr int UC = (2 * NTC + GRU_NW - 1) / GRU_NW;
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* const AL = fsm;            // d candidate rows [64][L1], then d gate rows [64][L2]
  float* const P = AL + 64 * L2;    // [2][64][RD] k-half partials
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g4 = lane >> 4, cl = lane & 15;
  float b1[UC][KS / 2], b2[UC][KS];  // unit u = w + 8 j: Wc_hᵀ and Wg_hᵀ fragments of column tile u % NTC, k half u / NTC
#pragma unroll
  for (int j = 0; j < UC; ++j) {
    const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
    const bool cu = u < 2 * NTC;
#pragma unroll
    for (int s = 0; s < KS / 2; ++s) b1[j][s] = cu ? Wch[(16 * ct + cl) * RD + 4 * (kh * KS / 2 + s) + g4] : 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) b2[j][s] = cu ? Wgh[(16 * ct + cl) * 2 * RD + 4 * (kh * KS + s) + g4] : 0.f;
  }
  float dh[EPT], dha[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + GRU_NT * i, n = e / RD;
    dh[i] = n < N ? dH[e] : 0.f;
  }
  for (int t = T2 - 1; t >= 0; --t) {
    int tq = tid;
    asm volatile("" : "+v"(tq));  // per-step element addresses recomputed, not hoisted (and spilled) across the loop
#pragma unroll
    for (int i = 0; i < EPT; ++i) {  // DCP = dh (1 - u)(1 - c²); DHA = dh u
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const long o = (long)t * N * RD + e;
        const float u = Uu[o], c = CC[o];
        const float dcp = dh[i] * (1.f - u) * (1.f - c * c);
        DCP[o] = dcp;
        AL[n * L1 + gru_perm(d, RD)] = dcp;
        dha[i] = dh[i] * u;
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int j = 0; j < UC; ++j) {
      const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
      if (u < 2 * NTC) {  // d(r·h) = DCP·Wc_hᵀ
        f32x4 acc[4] = {};
        gru_mm<KS / 2>(acc, AL, L1, KS, kh * KS / 2, b1[j], lane);
        gru_put(acc, P + kh * 64 * RD, RD, 16 * ct, lane);
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {  // DGP = [d(rh)·h·r(1-r), dh (h - c)·u(1-u)]; DHA += d(rh)·r
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const long o = (long)t * N * RD + e;
        const float h = HG[o], r = R[o], u = Uu[o], c = CC[o];
        const float drh = P[n * RD + d] + P[64 * RD + n * RD + d];
        const float gr = drh * h * r * (1.f - r), gu = dh[i] * (h - c) * u * (1.f - u);
        float* dg = DGP + ((long)t * N + n) * 2 * RD;
        dg[d] = gr;
        dg[RD + d] = gu;
        dha[i] += drh * r;
        AL[n * L2 + gru_perm(d, 2 * RD)] = gr;
        AL[n * L2 + gru_perm(RD + d, 2 * RD)] = gu;
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int j = 0; j < UC; ++j) {
      const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
      if (u < 2 * NTC) {  // d h(t) = DGP·Wg_hᵀ + DHA
        f32x4 acc[4] = {};
        gru_mm<KS>(acc, AL, L2, 2 * KS, kh * KS, b2[j], lane);
        gru_put(acc, P + kh * 64 * RD, RD, 16 * ct, lane);
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      dh[i] = n < N ? (P[n * RD + d] + P[64 * RD + n * RD + d]) + dha[i] : 0.f;
    }
    gru_lds_bar();
  }
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + GRU_NT * i, n = e / RD;
    if (n < N) dH[e] = dh[i];
  }
}
// bf16-operand forms for the bf16 training step (the per-step GEMMs they replace round A and B to
// bf16 too): v_mfma_f32_16x16x32_bf16, the A operands as bf16 rows in LDS (k contiguous: a lane's 8
// k of a k-step are one 16-byte read), B fragments 8 bf16 per lane per 32-deep k-step (half the fp32
// fragments' registers, which leaves room for the step's XG slice to be loaded before the products)
typedef __bf16 gru_bf8 __attribute__((ext_vector_type(8)));
template <int NKS>
__device__ __forceinline__ void gru_mm_bf(f32x4 (&acc)[4], const __bf16* AL, int ld, int k0, const gru_bf8 (&bf)[NKS],
                                          int lane) {
  const int r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    gru_bf8 a[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) a[mt] = *reinterpret_cast<const gru_bf8*>(AL + (16 * mt + r) * ld + k0 + 32 * ks + 8 * g);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], bf[ks], acc[mt], 0, 0, 0);
  }
}
// B fragment of a row-major fp32 W (row stride ldw): W[k0 + 32 ks + 8 g + e][col], e < 8, as bf16
__device__ __forceinline__ gru_bf8 gru_bfrag(const float* W, long ldw, int k, int col, bool on) {
  gru_bf8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (__bf16)(on ? W[(long)(k + e) * ldw + col] : 0.f);
  return v;
}

template <int RD>
__global__ __launch_bounds__(GRU_NT) void k_fe_gru_fwd_seq_bf(const float* __restrict__ XG, const float* __restrict__ Wgh,
                                                             const float* __restrict__ Wch, int N, int T2,
                                                             float* __restrict__ R, float* __restrict__ Uo,
                                                             float* __restrict__ RHo, float* __restrict__ CC,
                                                             float* __restrict__ HG) {
  constexpr int NTG = 2 * RD / 16, NTC = RD / 16, EPT = 64 * RD / GRU_NT, LB = RD + 8;
  constexpr int UG = (NTG + GRU_NW - 1) / GRU_NW, UC = (2 * NTC + GRU_NW - 1) / GRU_NW, KG = RD / 32, KC = RD / 64;
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* const h32 = fsm;                                           // h(t) [64][RD] fp32 (the state)
  __bf16* const hB = reinterpret_cast<__bf16*>(h32 + 64 * RD);      // bf16(h) rows [64][LB]
  __bf16* const rB = hB + 64 * LB;                                  // bf16(r·h) rows
  float* const P = reinterpret_cast<float*>(rB + 64 * LB);          // GG [64][2RD], then GC halves [2][64][RD]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g4 = lane >> 4, cl = lane & 15;
  gru_bf8 bg[UG][KG], bc[UC][KC];
#pragma unroll
  for (int j = 0; j < UG; ++j)
#pragma unroll
    for (int ks = 0; ks < KG; ++ks)
      bg[j][ks] = gru_bfrag(Wgh, 2 * RD, 32 * ks + 8 * g4, 16 * (w + GRU_NW * j) + cl, w + GRU_NW * j < NTG);
#pragma unroll
  for (int j = 0; j < UC; ++j) {
    const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
#pragma unroll
    for (int ks = 0; ks < KC; ++ks) bc[j][ks] = gru_bfrag(Wch, RD, kh * RD / 2 + 32 * ks + 8 * g4, 16 * ct + cl, u < 2 * NTC);
  }
  for (int e = tid; e < 64 * RD + 64 * LB; e += GRU_NT) fsm[e] = 0.f;  // h(0) = 0 (fp32 and the bf16 rows)
  float uu[EPT];
  __syncthreads();
  for (int t = 0; t < T2; ++t) {
    int tq = tid;
    asm volatile("" : "+v"(tq));
    float xr[EPT];  // this step's r-gate inputs, loaded ahead of the products
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      xr[i] = XG[((long)(n < N ? n : 0) * T2 + t) * 3 * RD + d];
    }
#pragma unroll
    for (int j = 0; j < UG; ++j)
      if (w + GRU_NW * j < NTG) {
        f32x4 acc[4] = {};
        gru_mm_bf<KG>(acc, hB, LB, 0, bg[j], lane);
        gru_put(acc, P, 2 * RD, 16 * (w + GRU_NW * j), lane);
      }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const float r = fe_sig(xr[i] + P[n * 2 * RD + d]);
        const float u = fe_sig(XG[((long)n * T2 + t) * 3 * RD + RD + d] + P[n * 2 * RD + RD + d]);
        const long o = ((long)t * N + n) * RD + d;
        const float rh = r * h32[n * RD + d];
        R[o] = r;
        Uo[o] = u;
        RHo[o] = rh;
        rB[n * LB + d] = (__bf16)rh;
        uu[i] = u;
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int j = 0; j < UC; ++j) {
      const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
      if (u < 2 * NTC) {
        f32x4 acc[4] = {};
        gru_mm_bf<KC>(acc, rB, LB, kh * RD / 2, bc[j], lane);
        gru_put(acc, P + kh * 64 * RD, RD, 16 * ct, lane);
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const float c = tanhf(XG[((long)n * T2 + t) * 3 * RD + 2 * RD + d] + (P[n * RD + d] + P[64 * RD + n * RD + d]));
        const long o = ((long)t * N + n) * RD + d;
        const float hn = uu[i] * h32[n * RD + d] + (1.f - uu[i]) * c;
        CC[o] = c;
        HG[o + (long)N * RD] = hn;
        h32[n * RD + d] = hn;
        hB[n * LB + d] = (__bf16)hn;
      }
    }
    gru_lds_bar();
  }
}

template <int RD>
__global__ __launch_bounds__(GRU_NT) void k_fe_gru_bwd_seq_bf(const float* __restrict__ Wgh, const float* __restrict__ Wch,
                                                             const float* __restrict__ R, const float* __restrict__ Uu,
                                                             const float* __restrict__ CC, const float* __restrict__ HG,
                                                             int N, int T2, float* __restrict__ dH,
                                                             float* __restrict__ DCP, float* __restrict__ DGP) {
  constexpr int NTC = RD / 16, EPT = 64 * RD / GRU_NT, L1 = RD + 8, L2 = 2 * RD + 8;
  constexpr int UC = (2 * NTC + GRU_NW - 1) / GRU_NW, K1 = RD / 64, K2 = RD / 32;
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  __bf16* const AB = reinterpret_cast<__bf16*>(fsm);                // bf16 d candidate rows [64][L1], then d gate rows [64][L2]
  float* const P = fsm + 64 * L2 / 2;                               // [2][64][RD] k-half partials
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g4 = lane >> 4, cl = lane & 15;
  gru_bf8 b1[UC][K1], b2[UC][K2];  // unit u: Wc_hᵀ / Wg_hᵀ fragments of column tile u % NTC, k half u / NTC
#pragma unroll
  for (int j = 0; j < UC; ++j) {
    const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
    const bool on = u < 2 * NTC;
#pragma unroll
    for (int ks = 0; ks < K1; ++ks) {  // Wc_hᵀ[k][col] = Wc_h[col][k]: k contiguous in the source row
      gru_bf8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)(on ? Wch[(long)(16 * ct + cl) * RD + kh * RD / 2 + 32 * ks + 8 * g4 + e] : 0.f);
      b1[j][ks] = v;
    }
#pragma unroll
    for (int ks = 0; ks < K2; ++ks) {
      gru_bf8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)(on ? Wgh[(long)(16 * ct + cl) * 2 * RD + kh * RD + 32 * ks + 8 * g4 + e] : 0.f);
      b2[j][ks] = v;
    }
  }
  float dh[EPT], dha[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + GRU_NT * i, n = e / RD;
    dh[i] = n < N ? dH[e] : 0.f;
  }
  for (int t = T2 - 1; t >= 0; --t) {
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const long o = (long)t * N * RD + e;
        const float u = Uu[o], c = CC[o];
        const float dcp = dh[i] * (1.f - u) * (1.f - c * c);
        DCP[o] = dcp;
        AB[n * L1 + d] = (__bf16)dcp;
        dha[i] = dh[i] * u;
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int j = 0; j < UC; ++j) {
      const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
      if (u < 2 * NTC) {
        f32x4 acc[4] = {};
        gru_mm_bf<K1>(acc, AB, L1, kh * RD / 2, b1[j], lane);
        gru_put(acc, P + kh * 64 * RD, RD, 16 * ct, lane);
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      if (n < N) {
        const long o = (long)t * N * RD + e;
        const float h = HG[o], r = R[o], u = Uu[o], c = CC[o];
        const float drh = P[n * RD + d] + P[64 * RD + n * RD + d];
        const float gr = drh * h * r * (1.f - r), gu = dh[i] * (h - c) * u * (1.f - u);
        float* dg = DGP + ((long)t * N + n) * 2 * RD;
        dg[d] = gr;
        dg[RD + d] = gu;
        dha[i] += drh * r;
        AB[n * L2 + d] = (__bf16)gr;
        AB[n * L2 + RD + d] = (__bf16)gu;
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int j = 0; j < UC; ++j) {
      const int u = w + GRU_NW * j, ct = u % NTC, kh = u / NTC;
      if (u < 2 * NTC) {
        f32x4 acc[4] = {};
        gru_mm_bf<K2>(acc, AB, L2, kh * RD, b2[j], lane);
        gru_put(acc, P + kh * 64 * RD, RD, 16 * ct, lane);
      }
    }
    gru_lds_bar();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tq + GRU_NT * i, n = e / RD, d = e % RD;
      dh[i] = n < N ? (P[n * RD + d] + P[64 * RD + n * RD + d]) + dha[i] : 0.f;
    }
    gru_lds_bar();
  }
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + GRU_NT * i, n = e / RD;
    if (n < N) dH[e] = dh[i];
  }
}

bool fe_gru_seq_ok(int N, int RD) { return N >= 1 && N <= 64 && (RD == 32 || RD == 128); }
static size_t fe_gru_lds(int RD, bool bwd) {
  return sizeof(float) * (bwd ? (size_t)64 * (2 * RD + 4) + 2 * 64 * RD : (size_t)2 * 64 * (RD + 4) + 64 * 2 * RD);
}
static size_t fe_gru_lds_bf(int RD, bool bwd) {
  return bwd ? (size_t)64 * (2 * RD + 8) * 2 + sizeof(float) * 2 * 64 * RD
             : sizeof(float) * (size_t)64 * RD + (size_t)2 * 64 * (RD + 8) * 2 + sizeof(float) * 64 * 2 * RD;
}
static void fe_gru_attrs() {
  static bool attr = false;
  if (attr) return;
  for (const void* k : {reinterpret_cast<const void*>(k_fe_gru_fwd_seq<32>), reinterpret_cast<const void*>(k_fe_gru_fwd_seq<128>),
                        reinterpret_cast<const void*>(k_fe_gru_bwd_seq<32>), reinterpret_cast<const void*>(k_fe_gru_bwd_seq<128>),
                        reinterpret_cast<const void*>(k_fe_gru_fwd_seq_bf<128>), reinterpret_cast<const void*>(k_fe_gru_bwd_seq_bf<128>)})
    TT2_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  attr = true;
}
void fe_gru_fwd_seq(const float* XG, const float* Wgh, const float* Wch, int N, int T2, int RD, float* R, float* Uu,
                    float* RH, float* CC, float* HG, hipStream_t s, bool bf16) {
  if (bf16 && RD == 128) {  // (a 32-deep bf16 k-step is deeper than RD = 32's k halves: fp32 form there)
    TT2_CHECK(fe_gru_seq_ok(N, RD), TT2_ERR_SHAPE_MISMATCH, "gru_fwd_seq: batch <= 64");
    fe_gru_attrs();
    hipLaunchKernelGGL(k_fe_gru_fwd_seq_bf<128>, dim3(1), dim3(GRU_NT), fe_gru_lds_bf(128, false), s, XG, Wgh, Wch, N, T2, R, Uu, RH, CC, HG);
    TT2_HIP(hipGetLastError());
    return;
  }
  TT2_CHECK(fe_gru_seq_ok(N, RD), TT2_ERR_SHAPE_MISMATCH, "gru_fwd_seq: batch <= 64, reference_depth 32 or 128");
  static bool attr = false;
  if (!attr) {
    for (const void* k : {reinterpret_cast<const void*>(k_fe_gru_fwd_seq<32>), reinterpret_cast<const void*>(k_fe_gru_fwd_seq<128>),
                          reinterpret_cast<const void*>(k_fe_gru_bwd_seq<32>), reinterpret_cast<const void*>(k_fe_gru_bwd_seq<128>)})
      TT2_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  if (RD == 128)
    hipLaunchKernelGGL(k_fe_gru_fwd_seq<128>, dim3(1), dim3(GRU_NT), fe_gru_lds(128, false), s, XG, Wgh, Wch, N, T2, R, Uu, RH, CC, HG);
  else
    hipLaunchKernelGGL(k_fe_gru_fwd_seq<32>, dim3(1), dim3(GRU_NT), fe_gru_lds(32, false), s, XG, Wgh, Wch, N, T2, R, Uu, RH, CC, HG);
  TT2_HIP(hipGetLastError());
}
void fe_gru_bwd_seq(const float* Wgh, const float* Wch, const float* R, const float* Uu, const float* CC, const float* HG,
                    int N, int T2, int RD, float* dH, float* DCP, float* DGP, hipStream_t s, bool bf16) {
  if (bf16 && RD == 128) {
    TT2_CHECK(fe_gru_seq_ok(N, RD), TT2_ERR_SHAPE_MISMATCH, "gru_bwd_seq: batch <= 64");
    fe_gru_attrs();
    hipLaunchKernelGGL(k_fe_gru_bwd_seq_bf<128>, dim3(1), dim3(GRU_NT), fe_gru_lds_bf(128, true), s, Wgh, Wch, R, Uu, CC, HG, N, T2, dH, DCP, DGP);
    TT2_HIP(hipGetLastError());
    return;
  }
  TT2_CHECK(fe_gru_seq_ok(N, RD), TT2_ERR_SHAPE_MISMATCH, "gru_bwd_seq: batch <= 64, reference_depth 32 or 128");
  static bool attr = false;
  if (!attr) {
    for (const void* k : {reinterpret_cast<const void*>(k_fe_gru_fwd_seq<32>), reinterpret_cast<const void*>(k_fe_gru_fwd_seq<128>),
                          reinterpret_cast<const void*>(k_fe_gru_bwd_seq<32>), reinterpret_cast<const void*>(k_fe_gru_bwd_seq<128>)})
      TT2_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  if (RD == 128)
    hipLaunchKernelGGL(k_fe_gru_bwd_seq<128>, dim3(1), dim3(GRU_NT), fe_gru_lds(128, true), s, Wgh, Wch, R, Uu, CC, HG, N, T2, dH, DCP, DGP);
  else
    hipLaunchKernelGGL(k_fe_gru_bwd_seq<32>, dim3(1), dim3(GRU_NT), fe_gru_lds(32, true), s, Wgh, Wch, R, Uu, CC, HG, N, T2, dH, DCP, DGP);
  TT2_HIP(hipGetLastError());
}

void fe_gru_a(const float* XG, const float* GG, const float* HG, int N, int T2, int D, int t, float* R, float* Uu,
              float* RH, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gru_a, dim3(fe_blk((long)N * D)), dim3(256), 0, s, XG, GG, HG, N, T2, D, t, R, Uu, RH);
}
void fe_gru_b(const float* XG, const float* GC, const float* Uu, int N, int T2, int D, int t, float* CC, float* HG,
              hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gru_b, dim3(fe_blk((long)N * D)), dim3(256), 0, s, XG, GC, Uu, N, T2, D, t, CC, HG);
}
// backward a: dh = dH; du = dh (h - c); dc = dh (1 - u); DCP = dc (1 - c^2); DHA = dh u
__global__ void k_fe_gru_bwd_a(const float* __restrict__ dH, const float* __restrict__ Uu, const float* __restrict__ CC,
                               const float* __restrict__ HG, int N, int D, int t, float* __restrict__ DCP,
                               float* __restrict__ DHA) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const long o = (long)t * N * D + i;
  const float dh = dH[i], u = Uu[o], c = CC[o];
  DCP[o] = dh * (1.f - u) * (1.f - c * c);
  DHA[i] = dh * u;
}
// backward b: dr = d(rh)·h; DHA += d(rh)·r; DGP = [dr r(1-r), du u(1-u)]
__global__ void k_fe_gru_bwd_b(const float* __restrict__ DRH, const float* __restrict__ R, const float* __restrict__ Uu,
                               const float* __restrict__ HG, const float* __restrict__ CC, const float* __restrict__ dH,
                               int N, int D, int t, float* __restrict__ DGP, float* __restrict__ DHA) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const int n = i / D, d = i % D;
  const long o = (long)t * N * D + i;
  const float h = HG[o], r = R[o], u = Uu[o], c = CC[o];
  const float drh = DRH[i];
  const float du = dH[i] * (h - c);
  float* dg = DGP + ((long)t * N + n) * 2 * D;
  dg[d] = drh * h * r * (1.f - r);
  dg[D + d] = du * u * (1.f - u);
  DHA[i] += drh * r;
}
void fe_gru_bwd_a(const float* dH, const float* Uu, const float* CC, const float* HG, int N, int D, int t, float* DCP,
                  float* DHA, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gru_bwd_a, dim3(fe_blk((long)N * D)), dim3(256), 0, s, dH, Uu, CC, HG, N, D, t, DCP, DHA);
}
void fe_gru_bwd_b(const float* DRH, const float* R, const float* Uu, const float* HG, const float* CC, const float* dH,
                  int N, int D, int t, float* DGP, float* DHA, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gru_bwd_b, dim3(fe_blk((long)N * D)), dim3(256), 0, s, DRH, R, Uu, HG, CC, dH, N, D, t, DGP,
                     DHA);
}
__global__ void k_fe_gru_dxg(const float* __restrict__ DGP, const float* __restrict__ DCP, int N, int T2, int D,
                             float* __restrict__ DXG) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * T2 * 3 * D) return;
  const int col = (int)(i % (3 * D));
  const long nt = i / (3 * D);
  const int t = (int)(nt % T2), n = (int)(nt / T2);
  DXG[i] = col < 2 * D ? DGP[((long)t * N + n) * 2 * D + col] : DCP[((long)t * N + n) * D + col - 2 * D];
}
void fe_gru_dxg(const float* DGP, const float* DCP, int N, int T2, int D, float* DXG, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gru_dxg, dim3(fe_blk((long)N * T2 * 3 * D)), dim3(256), 0, s, DGP, DCP, N, T2, D, DXG);
}
__global__ void k_fe_tanh_bwd(const float* __restrict__ dy, const float* __restrict__ y, long n,
                              float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = dy[i] * (1.f - y[i] * y[i]);
}
void fe_tanh_bwd(const float* dy, const float* y, long n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_tanh_bwd, dim3(fe_blk(n)), dim3(256), 0, s, dy, y, n, out);
}

// ---- GST --------------------------------------------------------------------------------------
// LDS of one row: q [A], kk [ntok][A], val [ntok][tokd] (= tanh(tokens)), nv [A/heads], w [heads][ntok]
constexpr int FE_GST_LDS = 128 + 16 * 128 + 16 * 64 + 32 + 4 * 16 + 64;

__device__ void fe_gst_common(const FeGst& a, int n, float* q, float* kk, float* val, float* nv, float* w) {
  const int tid = threadIdx.x, A = a.A, dh = A / a.heads;
  for (int i = tid; i < a.ntok * a.tokd; i += blockDim.x) val[i] = tanhf(a.tokens[i]);
  __syncthreads();
  for (int i = tid; i < A; i += blockDim.x) {
    float s = a.bq[i];
    for (int k = 0; k < a.refd; ++k) s += a.ref[(long)n * a.refd + k] * a.wq[(long)k * A + i];
    q[i] = s;
  }
  for (int i = tid; i < a.ntok * A; i += blockDim.x) {
    const int j = i / A, c = i % A;
    float s = a.bk[c];
    for (int k = 0; k < a.tokd; ++k) s += val[j * a.tokd + k] * a.wk[(long)k * A + c];
    kk[i] = s;
  }
  if (tid == 0) {  // normed_v = g v / ||v|| (multihead_attention.py:110-112)
    float ss = 0.f;
    for (int d = 0; d < dh; ++d) ss += a.v[d] * a.v[d];
    const float sc = a.g[0] / sqrtf(ss);
    for (int d = 0; d < dh; ++d) nv[d] = sc * a.v[d];
  }
  __syncthreads();
  if (tid < a.heads * a.ntok) {  // scores and softmax over tokens, per head
    const int h = tid / a.ntok, j = tid % a.ntok;
    float s = 0.f;
    for (int d = 0; d < dh; ++d) s += nv[d] * tanhf(kk[j * A + h * dh + d] + q[h * dh + d] + a.bb[d]);
    w[tid] = s;
  }
  __syncthreads();
  if (tid < a.heads) {
    float mx = -INFINITY, sum = 0.f;
    for (int j = 0; j < a.ntok; ++j) mx = fmaxf(mx, w[tid * a.ntok + j]);
    for (int j = 0; j < a.ntok; ++j) sum += expf(w[tid * a.ntok + j] - mx);
    for (int j = 0; j < a.ntok; ++j) w[tid * a.ntok + j] = expf(w[tid * a.ntok + j] - mx) / sum;
  }
  __syncthreads();
}

__global__ void k_fe_gst_fwd(FeGst a) {
  extern __shared__ float sm[];
  float* q = sm; float* kk = q + 128; float* val = kk + 16 * 128; float* nv = val + 16 * 64; float* w = nv + 32;
  const int n = blockIdx.x;
  fe_gst_common(a, n, q, kk, val, nv, w);
  for (int i = threadIdx.x; i < a.heads * a.tokd; i += blockDim.x) {  // context over tiled values
    const int h = i / a.tokd, e = i % a.tokd;
    float s = 0.f;
    for (int j = 0; j < a.ntok; ++j) s += w[h * a.ntok + j] * val[j * a.tokd + e];
    a.style[(long)n * a.style_ld + a.style_off + i] = s;
  }
}
void fe_gst_fwd(const FeGst& a, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gst_fwd, dim3(a.N), dim3(256), sizeof(float) * FE_GST_LDS, s, a);
}

__global__ void k_fe_gst_bwd(FeGst a) {
  extern __shared__ float sm[];
  float* q = sm; float* kk = q + 128; float* val = kk + 16 * 128; float* nv = val + 16 * 64; float* w = nv + 32;
  float* dw = w + 64;  // [heads][ntok], then ds
  const int n = blockIdx.x, tid = threadIdx.x, A = a.A, dh = A / a.heads;
  fe_gst_common(a, n, q, kk, val, nv, w);
  const float* dout = a.dstyle + (long)n * a.style_ld + a.style_off;
  if (tid < a.heads * a.ntok) {  // d w[h][j] = Σ_e dout[h][e] val[j][e]
    const int h = tid / a.ntok, j = tid % a.ntok;
    float s = 0.f;
    for (int e = 0; e < a.tokd; ++e) s += dout[h * a.tokd + e] * val[j * a.tokd + e];
    dw[tid] = s;
  }
  __syncthreads();
  if (tid < a.heads) {  // softmax backward: ds = w (dw - Σ w dw)
    float s = 0.f;
    for (int j = 0; j < a.ntok; ++j) s += w[tid * a.ntok + j] * dw[tid * a.ntok + j];
    for (int j = 0; j < a.ntok; ++j) dw[tid * a.ntok + j] = w[tid * a.ntok + j] * (dw[tid * a.ntok + j] - s);
  }
  __syncthreads();
  // value path: d val[j][e] = Σ_h w[h][j] dout[h][e]
  for (int i = tid; i < a.ntok * a.tokd; i += blockDim.x) {
    const int j = i / a.tokd, e = i % a.tokd;
    float s = 0.f;
    for (int h = 0; h < a.heads; ++h) s += w[h * a.ntok + j] * dout[h * a.tokd + e];
    a.pdv[(long)n * a.ntok * a.tokd + i] = s;
  }
  // d pre[h][j][d] = ds[h][j] nv[d] (1 - th^2): d kk, d q, d bb, d nv
  for (int i = tid; i < a.ntok * A; i += blockDim.x) {
    const int j = i / A, c = i % A, h = c / dh, d = c % dh;
    const float th = tanhf(kk[i] + q[c] + a.bb[d]);
    a.pdkk[(long)n * a.ntok * A + i] = dw[h * a.ntok + j] * nv[d] * (1.f - th * th);
  }
  for (int c = tid; c < A; c += blockDim.x) {
    const int h = c / dh, d = c % dh;
    float s = 0.f;
    for (int j = 0; j < a.ntok; ++j) {
      const float th = tanhf(kk[j * A + c] + q[c] + a.bb[d]);
      s += dw[h * a.ntok + j] * nv[d] * (1.f - th * th);
    }
    a.dq[(long)n * A + c] = s;
  }
  for (int d = tid; d < dh; d += blockDim.x) {
    float snv = 0.f, sbb = 0.f;
    for (int h = 0; h < a.heads; ++h)
      for (int j = 0; j < a.ntok; ++j) {
        const float th = tanhf(kk[j * A + h * dh + d] + q[h * dh + d] + a.bb[d]);
        snv += dw[h * a.ntok + j] * th;
        sbb += dw[h * a.ntok + j] * nv[d] * (1.f - th * th);
      }
    a.pdnv[(long)n * dh + d] = snv;
    a.pdbb[(long)n * dh + d] = sbb;
  }
}
void fe_gst_bwd(const FeGst& a, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gst_bwd, dim3(a.N), dim3(256), sizeof(float) * (FE_GST_LDS + 64), s, a);
}

// one block: d Wk = valᵀ·dkk, d bk = Σ_j dkk, d val += dkk·Wkᵀ, d tokens = d val (1 - val^2),
// d v / d g through normed_v = g v / ||v||, d attention_b
__global__ void k_fe_gst_final(FeGst a, const float* __restrict__ dkk, const float* __restrict__ dval,
                               const float* __restrict__ dnv, const float* __restrict__ dbb, float* __restrict__ dwk,
                               float* __restrict__ dbk, float* __restrict__ dtok, float* __restrict__ dv,
                               float* __restrict__ dg, float* __restrict__ dbbo) {
  const int tid = threadIdx.x, A = a.A, dh = A / a.heads;
  for (int i = tid; i < a.tokd * A; i += blockDim.x) {
    const int e = i / A, c = i % A;
    float s = 0.f;
    for (int j = 0; j < a.ntok; ++j) s += tanhf(a.tokens[j * a.tokd + e]) * dkk[j * A + c];
    dwk[i] = s;
  }
  for (int c = tid; c < A; c += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < a.ntok; ++j) s += dkk[j * A + c];
    dbk[c] = s;
  }
  for (int i = tid; i < a.ntok * a.tokd; i += blockDim.x) {
    const int j = i / a.tokd, e = i % a.tokd;
    float s = dval[i];
    for (int c = 0; c < A; ++c) s += dkk[j * A + c] * a.wk[(long)e * A + c];
    const float vt = tanhf(a.tokens[i]);
    dtok[i] = s * (1.f - vt * vt);
  }
  if (tid == 0) {
    float ss = 0.f, vd = 0.f;
    for (int d = 0; d < dh; ++d) {
      ss += a.v[d] * a.v[d];
      vd += a.v[d] * dnv[d];
    }
    const float nrm = sqrtf(ss), g = a.g[0];
    dg[0] = vd / nrm;
    for (int d = 0; d < dh; ++d) dv[d] = g * (dnv[d] / nrm - a.v[d] * vd / (nrm * nrm * nrm));
    for (int d = 0; d < dh; ++d) dbbo[d] = dbb[d];
  }
}
void fe_gst_final(const FeGst& a, const float* dkk, const float* dval, const float* dnv, const float* dbb, float* dwk,
                  float* dbk, float* dtok, float* dv, float* dg, float* dbbo, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_gst_final, dim3(1), dim3(256), 0, s, a, dkk, dval, dnv, dbb, dwk, dbk, dtok, dv, dg, dbbo);
}

// ---- memory ---------------------------------------------------------------------------------------
__global__ void k_fe_memory(const float* __restrict__ ENC, const float* __restrict__ STY, int B, int T, int E2,
                            int SW, float* __restrict__ MEM) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int D = E2 + SW;
  if (i >= (long)B * T * D) return;
  const int d = (int)(i % D);
  const long bt = i / D;
  const int b = (int)(bt / T);
  MEM[i] = d < E2 ? ENC[bt * E2 + d] : STY[(long)b * SW + d - E2];
}
void fe_memory(const float* ENC, const float* STY, int B, int T, int E2, int SW, float* MEM, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_memory, dim3(fe_blk((long)B * T * (E2 + SW))), dim3(256), 0, s, ENC, STY, B, T, E2, SW, MEM);
}
__global__ void k_fe_style_grad(const float* __restrict__ DMEM, int B, int T, int D, int E2, float* __restrict__ DSTY) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int SW = D - E2;
  if (i >= B * SW) return;
  const int b = i / SW, c = i % SW;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += DMEM[((long)b * T + t) * D + E2 + c];
  DSTY[i] = s;
}
void fe_style_grad(const float* DMEM, int B, int T, int D, int E2, float* DSTY, hipStream_t s) {
  hipLaunchKernelGGL(k_fe_style_grad, dim3(fe_blk((long)B * (D - E2))), dim3(256), 0, s, DMEM, B, T, D, E2, DSTY);
}

}  // namespace tt2
