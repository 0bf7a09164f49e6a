// Persistent BPTT backward of the teacher-forced decoder (train_bwd_persist.h).
//
// Why: the per-step backward of train.hip is four launches per decoder step (attention backward,
// LSTM-2 cell backward behind d query·Wq^T, [d h1 | d hz2] = dG2·W2^T + LSTM-1 cell backward, d X1 =
// dG1·W1^T): 49.5 us per step, the bf16 values and the LSTM weights re-streamed from the MALL every
// step.  Here one launch walks t = T-1 .. 0 with them resident.
//
// Roles of work-group g (all 256 have all three):
//   attention  row rb = g & 63, quarter s = g >> 6: context channels [256 s, 256 s + 256) (the bf16
//              values quarter as MFMA A fragments in AGPRs) and attention dims [32 s, 32 s + 32)
//              (th, du, d keys, the query columns of the d h2 product, the location-conv backward)
//   unit       hidden units [4g, 4g + 4) of both layers, all 64 rows: the LSTM cell backward
//              (k_tr_lstm_bwd's arithmetic), the carried d c and the zoneout residuals in registers
//   product    K-block kb = g >> 4 (units [64 kb, 64 kb + 64) x 4 gates = 256 gate columns, the
//              tb_kperm order) x N-block nb = g & 15 (outputs [128 nb, 128 nb + 128) of 2048) of both
//              K = 4096 products, [d h1 | d hz2_{t-1}] = dG2·W2^T and [d ctx_{t-1} | d hz1_{t-1}] =
//              dG1·W1^T: the 2 x 64 KB bf16 weight blocks register-resident, partials per K-block
//
// One step t (tag T - t, exchange buffers by parity t & 1):
//   ATT  wave w waits the P1 partials of step t+1 for its 64 channels, d ctx = d PIN + Σ_kb P1;
//        d align partial = values quarter · d ctx (hi / lo bf16 halves of d ctx: ~fp32 products) +
//        this quarter's running d cum partial -> granules to the other 3 quarters; take and sum them in
//        quarter order (identical in all four); softmax backward; du = de·v_a·(1 - th²) of the own dims;
//        d query of the own dims (complete) -> DQ and d h2 partial = dq·Wq[:, own dims]^T -> QX
//   CELL2  wait QX of every (row, quarter), d h2 = d PIN + Σ_s QX; d hz2 = Σ_kb P2_{t+1} + residual;
//        cell backward -> dG2 (fp32 slot + bf16 exchange)
//   PROD2  wait the K-block's 16 unit producers, dG2 block · W2 block -> P2
//   CELL1  wait P2 of the own N-block, d h1 = Σ_kb P2; d hz1 = Σ_kb P1_{t+1} + residual; cell
//        backward -> dG1
//   PROD1  wait the K-block's dG1, dG1 block · W1 block -> P1 (consumed at step t-1)
// Off the chain, after QX is published: G[tap][a] += Σ_j cum_t[j + tap - 15]·du[j][a] (d W_loc, d Kc,
// d bc after the launch) and the location-conv backward into this quarter's d cum partial
// (M = du·KW^T over the own dims, then the tap diagonals).
// Exchange protocol as train_persist.hip: sc1 write-through stores, drained before one barrier and the
// flag stores (8 replicas), sc1 loads by waves that polled the producers or joined a barrier behind
// such polls; the d align partials are data-tagged granules.  Spins are bounded (2 s).
#include "tp_device.h"

#include "train_bwd_persist.h"

namespace tt2 {

enum { TB_PH_P1 = 0, TB_PH_Q = 1, TB_PH_G2 = 2, TB_PH_P2 = 3, TB_PH_G1 = 4, TB_PH_E = 5 };
constexpr int TB_NW = TP_NT / 64;        // waves
constexpr int TB_TM = TP_TMAX;           // encoder positions (capacity)
constexpr int TB_NPT = TB_TM / 16;       // position tiles
constexpr int TB_PTW = TB_NPT / TB_NW;   // position tiles per wave
constexpr int TB_K4 = 4 * TP_H;          // gate columns
static_assert(TB_NPT % TB_NW == 0 && TP_NT == 256 && TP_A == 128 && TP_D == 1024 && TP_H == 1024,
              "train_bwd_persist geometry");

// LDS layout (floats)
constexpr int TBL_DCTX = 0;                   // [256] d ctx of this quarter
constexpr int TBL_EP = TBL_DCTX + 256;        // [TM] own d align partial
constexpr int TBL_DA = TBL_EP + TB_TM;        // [TM] d align, then de
constexpr int TBL_DS = TBL_DA + TB_TM;        // [TM] running d cum partial of the own dims
constexpr int TBL_CUM = TBL_DS + TB_TM;       // [TM + 48] cum_t at +15, zero padded
constexpr int TBL_DU = TBL_CUM + TB_TM + 48;  // [TM][33] du of the own dims
constexpr int TBL_M = TBL_DU + TB_TM * 33;    // [TM][33] M[j][tap] = Σ_d du[j][d]·KW[d][tap]
constexpr int TBL_RED = TBL_M + TB_TM * 33;   // [2][TB_NW][32] wave partials of dq / d v_a
constexpr int TBL_DQ = TBL_RED + 2 * TB_NW * 32;  // [32] dq
constexpr int TBL_SC = TBL_DQ + 32;           // [16] reduction scratch, then ints
constexpr int TBL_WQ = TBL_SC + 32;           // [64 M-tiles][64 lanes] bf16 x 8: the own query columns
constexpr int TBL_END = TBL_WQ + 64 * 64 * 4;

size_t tb_lds_bytes() { return sizeof(float) * (size_t)TBL_END; }

__device__ __forceinline__ float tb_block_sum(float v, float* scr) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scr[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = scr[0];
#pragma unroll
  for (int i = 1; i < TB_NW; ++i) r += scr[i];
  return r;
}
// sum over the 16 lanes of each lane row (xor within the low 4 lane bits)
__device__ __forceinline__ float tb_row16_sum(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// wave poll of n producers, producer(l) for lane l < n (this XCD group's flag replica)
template <class F>
__device__ __forceinline__ bool tb_poll(const TbArgs& a, int ph, int n, unsigned tag, F producer) {
  const unsigned* f = a.flags + ((long)ph * TP_NREP + (blockIdx.x & (TP_NREP - 1))) * TP_NB;
  const int lane = threadIdx.x & 63;
  const int pidx = lane < n ? producer(lane) : 0;
  return tp_spin(a, ph, [&] { return lane >= n || tp_flag(f + pidx) >= tag; });
}
// 8 floats -> bf16 fragment (round to nearest even, as every bf16 operand of the step)
__device__ __forceinline__ tp_bf8 tb_bf8(const float (&x)[8]) {
  tp_bf8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (__bf16)x[e];
  return v;
}
__device__ __forceinline__ float tb_ld(const __amdgpu_buffer_rsrc_t rs, int byte_off) {  // sc1 dword load
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, byte_off, 0, 16));
}
__device__ __forceinline__ void tb_st(void* base, int byte_off, float v) {  // sc1 write-through dword store
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), tp_rsrc(base), byte_off, 0, 16);
}

// LSTM cell backward of one (row, unit) (k_tr_lstm_bwd / tf_cell_bwd): returns the 4 gate gradients,
// updates the carried d(zoned c) and returns the zoneout residual (1 - kh)·dhz in *res
struct TbCell {
  float g[4];  // activated gates i, j, f, o
  float cn, cp, kc, kh;
};
__device__ __forceinline__ void tb_cell_bwd(const TbCell& v, float dext, float dhz, float& dc, float& res, float (&d)[4]) {
  const float si = v.g[0], tj = v.g[1], sf = v.g[2], so = v.g[3];
  const float dhn = dext + v.kh * dhz;
  const float tc = tanhf(v.cn);
  const float dcn = v.kc * dc + dhn * so * (1.f - tc * tc);
  const float dso = dhn * tc, dsf = dcn * v.cp, dsi = dcn * tj, dtj = dcn * si;
  d[0] = dsi * si * (1.f - si);
  d[1] = dtj * (1.f - tj * tj);
  d[2] = dsf * sf * (1.f - sf);
  d[3] = dso * so * (1.f - so);
  dc = (1.f - v.kc) * dc + dcn * sf;
  res = (1.f - v.kh) * dhz;
}

__global__ __launch_bounds__(TP_NT, 1) void k_tr_bwd_persist(TbArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const dctx_s = sm + TBL_DCTX;
  float* const ep = sm + TBL_EP;
  float* const da_s = sm + TBL_DA;
  float* const ds = sm + TBL_DS;
  float* const cum_s = sm + TBL_CUM;
  float* const dus = sm + TBL_DU;
  float* const ms = sm + TBL_M;
  float* const red = sm + TBL_RED;
  float* const dq_s = sm + TBL_DQ;
  float* const scr = sm + TBL_SC;
  int* const sfail = reinterpret_cast<int*>(sm + TBL_SC + 16);
  constexpr int H = TP_H, D = TP_D, A = TP_A, P = TP_P, LX1 = TP_LX1, K4 = TB_K4, TM = TB_TM;
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int B = a.B, T = a.T, Tin = a.Tin;
  const int rb = g & 63, sq = g >> 6;  // attention row, quarter
  const bool arow = rb < B;
  const int kb = g >> 4, nb = g & 15;  // product K-block, N-block
  const int jl = lane & 15, g4 = lane >> 4;

  // ---- product weights, B fragments of v_mfma_f32_16x16x32_bf16: wave w owns the output columns
  // m = 128 nb + 32 w + 16 nt + jl; k-step ks of the K-block covers its exchange positions
  // 32 ks + 8 g4 + e -> gate column c = (p >> 6)·H + 64 kb + (p & 63)
  tp_bf8 w2f[2][8], w1f[2][8];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int m = 128 * nb + 32 * w + 16 * nt + jl;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int p0 = 32 * ks + 8 * g4;
      const int c0 = (p0 >> 6) * H + 64 * kb + (p0 & 63);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        w2f[nt][ks][e] = a.K2T[(long)(c0 + e) * 2 * H + m];       // W2[m][c]: m < H h1 rows, then hz2
        w1f[nt][ks][e] = a.K1T[(long)(c0 + e) * LX1 + P + m];     // W1[P + m][c]: ctx rows, then hz1
      }
    }
  }
  // ---- attention row constants
  // values quarter as A fragments (AGPRs): tile pt = w + 4 r, k-step ks: lane holds
  // values16[rb][16 pt + jl][256 sq + 32 ks + 8 g4 .. + 8]
  float vfr[TB_PTW][8][4];
#pragma unroll
  for (int r = 0; r < TB_PTW; ++r) {
    const int j = 16 * (w + 4 * r) + jl;
    const bool ok = arow && j < Tin;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const tp_u4 v = ok ? *reinterpret_cast<const tp_u4*>(a.values16 + ((long)rb * Tin + j) * D + 256 * sq + 32 * ks + 8 * g4)
                         : tp_u4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < 4; ++i) vfr[r][ks][i] = tp_aput(__uint_as_float(v[i]));
    }
  }
  // query columns of the own dims as A fragments of the d h2 product, in LDS: M-tile mt = 16 w + i
  // (rows u = 16 mt + jl), lane holds Wq[u][32 sq + 8 g4 .. + 8]
  tp_bf8* const wqf = reinterpret_cast<tp_bf8*>(sm + TBL_WQ);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int u = 16 * (16 * w + i) + jl;
    wqf[(16 * w + i) * 64 + lane] = arow ? *reinterpret_cast<const tp_bf8*>(a.Wq + (long)u * A + 32 * sq + 8 * g4) : tp_bf8{};
  }
  // KW^T as B fragments of the location-conv backward (v_mfma_f32_16x16x4f32): tap tile nt, k-step ks:
  // lane holds KW[dim 32 sq + 4 ks + g4][tap 16 nt + jl] (tap 31, the bias column, zero)
  float kwb[2][8];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int tap = 16 * nt + jl;
      kwb[nt][ks] = (arow && tap < 31) ? a.KWT[(32 * sq + 4 * ks + g4) * 32 + tap] : 0.f;
    }
  // v_a of the lane's dims 16 mt + 4 g4 + i (energy-tile layout, as the forward)
  float vav[8];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) vav[4 * mt + i] = a.va[32 * sq + 16 * mt + 4 * g4 + i];
  // accumulators: d keys of the lane's (position, dims) (AGPRs), d v_a / d b_a of dim tid < 32, G tile
  float dkey[TB_PTW][8];
#pragma unroll
  for (int r = 0; r < TB_PTW; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) dkey[r][i] = tp_aput(0.f);
  float dva = 0.f, dba = 0.f;
  tp_f4 gacc = {0.f, 0.f, 0.f, 0.f};
  const int len = arow ? a.lens[rb] : 0;
  for (int e = tid; e < TM + 48; e += TP_NT) cum_s[e] = 0.f;
  for (int e = tid; e < TM; e += TP_NT) ds[e] = 0.f;
  if (tid == 0) sfail[0] = 0;

  // unit role: thread (row er, unit en); carried d c of both layers and the zoneout residuals
  const int er = tid >> 2, eu = tid & 3, en = 4 * g + eu;
  const bool erow = er < B;
  const int evo = er * H + en;
  float dc1 = 0.f, dc2 = 0.f, rr1 = 0.f, rr2 = 0.f;
  __syncthreads();

#define TB_STAMP(i)                                                         \
  do {                                                                      \
    if (stp && tid == 0) stp[g * 32 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  for (int t = T - 1; t >= 0; --t) {
    const int par = t & 1, parn = par ^ 1;
    const unsigned tag = (unsigned)(T - t), tagn = tag - 1u;  // tagn: step t+1
    const bool first = t == T - 1;
    const long tb = (long)t * B;
    long long* const stp = t == a.stamp_step ? a.stamps : nullptr;
    asm volatile("" ::: "memory");
    TB_STAMP(0);
    // unit-role operands of one cell (layer 0 / 1), loaded ahead of that cell's waits
    auto cell_load = [&](int layer, TbCell& c, float& dpin) {
      if (!erow) return;
      const float* gg = (layer ? a.G2 : a.G1) + (tb + er) * K4 + en;
#pragma unroll
      for (int q = 0; q < 4; ++q) c.g[q] = gg[q * H];
      c.cn = (layer ? a.CN2 : a.CN1)[tb * H + evo];
      c.cp = (layer ? a.C2 : a.C1)[tb * H + evo];
      if (layer) dpin = a.dPIN[(tb + er) * (H + D) + en];
      if (a.zm) {
        const uint8_t* z = a.zm + (long)t * 4 * B * H + evo + (long)(2 * layer) * B * H;
        c.kc = (float)z[0];
        c.kh = (float)z[(long)B * H];
      } else {
        c.kc = c.kh = 1.f - a.z;
      }
    };
    // ================= ATT
    if (arow) {
      const long rt = (tb + rb) * Tin;  // this row's [Tin] block of step t
      const float aj = tid < Tin ? a.ALN[rt + tid] : 0.f;
      const float cumv = tid < Tin ? a.CUM[rt + tid] : 0.f;
      tp_f4 th[TB_PTW][2];
#pragma unroll
      for (int r = 0; r < TB_PTW; ++r) {
        const int j = 16 * (w + 4 * r) + jl;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          th[r][mt] = j < Tin ? *reinterpret_cast<const tp_f4*>(a.TH + (rt + j) * A + 32 * sq + 16 * mt + 4 * g4)
                              : tp_f4{0.f, 0.f, 0.f, 0.f};
      }
      // d ctx of channel 256 sq + tid = d PIN + Σ_kb P1_{t+1} (wave w: the N-block 2 sq + (w >> 1))
      float dctx = a.dPIN[(tb + rb) * (H + D) + H + 256 * sq + tid];
      if (!first) {
        const int nbw = 2 * sq + (w >> 1);
        if (!tb_poll(a, TB_PH_P1, TB_NKB, tagn, [&](int l) { return 16 * l + nbw; })) sfail[0] = 1;
        TB_STAMP(1);
        const auto rs = tp_rsrc(a.P1X + (long)parn * TB_NKB * 64 * TB_NOUT);
        float pv[TB_NKB];
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) pv[k] = tb_ld(rs, (int)((((long)k * 64 + rb) * TB_NOUT + 256 * sq + tid) * 4));
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) dctx += pv[k];
      }
      a.DCTX[(tb + rb) * D + 256 * sq + tid] = dctx;
      dctx_s[tid] = dctx;
      __syncthreads();
      TB_STAMP(2);
      if (sfail[0]) return;
      // d align partial of the own channels: values quarter · (hi, lo) bf16 halves of d ctx in the B
      // columns 0 / 1 of v_mfma_f32_16x16x32_bf16 (the other columns zero)
      {
        tp_bf8 bfr[8];
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          float x[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = dctx_s[32 * ks + 8 * g4 + e];
            const float hi = (float)(__bf16)v;
            x[e] = jl == 0 ? hi : jl == 1 ? v - hi : 0.f;
          }
          bfr[ks] = tb_bf8(x);
        }
#pragma unroll
        for (int r = 0; r < TB_PTW; ++r) {
          const int pt = w + 4 * r;
          if (16 * pt >= Tin) break;  // wave-uniform
          tp_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) {
            const tp_u4 u = {__float_as_uint(tp_aget(vfr[r][ks][0])), __float_as_uint(tp_aget(vfr[r][ks][1])),
                             __float_as_uint(tp_aget(vfr[r][ks][2])), __float_as_uint(tp_aget(vfr[r][ks][3]))};
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(tp_bf8, u), bfr[ks], acc, 0, 0, 0);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float lo = __shfl(acc[i], lane + 1, 64);
            const int j = 16 * pt + 4 * g4 + i;
            if (jl == 0 && j < Tin) ep[j] = acc[i] + lo + ds[j];
          }
        }
      }
      __syncthreads();
      // granules of the own partial, then the other quarters' (summed in quarter order)
      if (tid < Tin)
        __builtin_amdgcn_raw_buffer_store_b64(tp_u2{__float_as_uint(ep[tid]), tag},
                                              tp_rsrc(a.EX + (((long)par * 64 + rb) * 4 + sq) * TM), tid * 8, 0, 16);
      TB_STAMP(3);
      if (w < (Tin + 63) / 64) {
        const bool act = tid < Tin;
        const auto rs = tp_rsrc(a.EX + ((long)par * 64 + rb) * 4 * TM);
        float e4[4];
        const float own = act ? ep[tid] : 0.f;
        const bool ok = tp_spin(a, TB_PH_E, [&] {
          bool good = true;
          if (act) {
            unsigned bad = 0u;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              if (s == sq) {
                e4[s] = own;
              } else {
                const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (s * TM + tid) * 8, 0, 16);
                e4[s] = __uint_as_float(x[0]);
                bad |= x[1] ^ tag;
              }
            }
            good = bad == 0u;
          }
          return good;
        });
        if (!ok) sfail[0] = 1;
        if (act) da_s[tid] = ((e4[0] + e4[1]) + e4[2]) + e4[3];
      }
      __syncthreads();
      TB_STAMP(4);
      if (sfail[0]) return;
      // softmax backward (attention.py:218): de_j = a_j (d a_j - Σ_k a_k d a_k), 0 past the length
      const float dav = tid < Tin ? da_s[tid] : 0.f;
      const float ssum = tb_block_sum(aj * dav, scr);
      if (tid < Tin) da_s[tid] = tid < len ? aj * (dav - ssum) : 0.f;
      if (tid < Tin) cum_s[15 + tid] = cumv;
      __syncthreads();
      // du of the own dims (energy-tile layout): d keys, d query, d v_a; du -> LDS
      float dqp[8], dvp[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) dqp[i] = dvp[i] = 0.f;
#pragma unroll
      for (int r = 0; r < TB_PTW; ++r) {
        const int pt = w + 4 * r;
        if (16 * pt >= Tin) break;  // wave-uniform
        const int j = 16 * pt + jl;
        const float dej = j < Tin ? da_s[j] : 0.f;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float thv = th[r][mt][i];
            const float du = dej * vav[4 * mt + i] * (1.f - thv * thv);
            dkey[r][4 * mt + i] = tp_aput(tp_aget(dkey[r][4 * mt + i]) + du);
            dqp[4 * mt + i] += du;
            dvp[4 * mt + i] += dej * thv;
            dus[j * 33 + 16 * mt + 4 * g4 + i] = du;
          }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dqp[i] = tb_row16_sum(dqp[i]);
        dvp[i] = tb_row16_sum(dvp[i]);
      }
      if (jl == 0) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            red[w * 32 + 16 * mt + 4 * g4 + i] = dqp[4 * mt + i];
            red[TB_NW * 32 + w * 32 + 16 * mt + 4 * g4 + i] = dvp[4 * mt + i];
          }
      }
      __syncthreads();
      if (tid < 32) {
        float q = 0.f, v = 0.f;
#pragma unroll
        for (int ww = 0; ww < TB_NW; ++ww) {
          q += red[ww * 32 + tid];
          v += red[TB_NW * 32 + ww * 32 + tid];
        }
        dq_s[tid] = q;
        dba += q;
        dva += v;
        a.DQ[(tb + rb) * A + 32 * sq + tid] = q;
      }
      __syncthreads();
      TB_STAMP(5);
      // d h2 partial of this quarter: Σ_{own dims} Wq[u][a]·dq[a] for all u (bf16 operands as the
      // per-step product k_tr_fused<TF_BWD_H>), B column 0 = dq
      {
        float x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = jl == 0 ? dq_s[8 * g4 + e] : 0.f;
        const tp_bf8 bq = tb_bf8(x);
        float* const qrow = a.QX + (((long)par * 4 + sq) * 64 + rb) * H;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const tp_f4 acc =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(wqf[(16 * w + i) * 64 + lane], bq, tp_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          if (jl == 0) tp_st16(qrow, (16 * (16 * w + i) + 4 * g4) * 4, __builtin_bit_cast(tp_u4, acc));
        }
      }
      tp_publish(a, TB_PH_Q, tag);
      TB_STAMP(6);
      // ---- off the chain: d W_loc accumulators and the location-conv backward of the own dims
      {  // G^T[a][tap] += Σ_j du[j][a]·cum_t[j + tap - 15]: wave w -> dim tile w >> 1, tap tile w & 1
        const int mt = w >> 1, nt = w & 1;
        const int nks = (Tin + 3) >> 2;
        for (int ks = 0; ks < nks; ++ks) {
          const int j = 4 * ks + g4;
          gacc = __builtin_amdgcn_mfma_f32_16x16x4f32(dus[j * 33 + 16 * mt + jl], cum_s[j + 16 * nt + jl], gacc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int q6 = 0; q6 < 2 * TB_PTW; ++q6) {  // M tiles (position tile, tap tile) = w + 4 q6
        const int idx = w + 4 * q6, pt = idx >> 1, nt = idx & 1;
        if (16 * pt >= Tin) continue;  // wave-uniform
        tp_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dus[(16 * pt + jl) * 33 + 4 * ks + g4], kwb[nt][ks], acc, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) ms[(16 * pt + 4 * g4 + i) * 33 + 16 * nt + jl] = acc[i];
      }
      __syncthreads();
      if (tid < Tin) {  // d cum_t[i] += Σ_tap M[i - tap + 15][tap]
        float v = 0.f;
        for (int tap = 0; tap < 31; ++tap) {
          const int jj = tid - tap + 15;
          if (jj >= 0 && jj < Tin) v += ms[jj * 33 + tap];
        }
        ds[tid] += v;
      }
    }
    TB_STAMP(7);
    // ================= CELL2: d hz2 from step t+1's product, d h2 from the 4 quarters' QX
    TbCell c2{};
    float dpin_h = 0.f;
    cell_load(1, c2, dpin_h);
    float dhz2 = 0.f;
    if (!first) {
      if (!tb_poll(a, TB_PH_P2, TB_NKB, tagn, [&](int l) { return 16 * l + 8 + (g >> 5); })) sfail[0] = 1;
      if (erow) {
        const auto rs = tp_rsrc(a.P2X + (long)parn * TB_NKB * 64 * TB_NOUT);
        float pv[TB_NKB];
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) pv[k] = tb_ld(rs, (int)((((long)k * 64 + er) * TB_NOUT + H + en) * 4));
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) dhz2 += pv[k];
      }
      dhz2 += rr2;
    }
    if (!tb_poll(a, TB_PH_Q, B, tag, [&](int l) { return 64 * w + l; })) sfail[0] = 1;  // wave w: quarter w
    __syncthreads();  // every quarter's poll behind this barrier
    TB_STAMP(8);
    if (sfail[0]) return;
    {
      float d[4] = {0.f, 0.f, 0.f, 0.f};
      if (erow) {
        const auto rs = tp_rsrc(a.QX + (long)par * 4 * 64 * H);
        float qv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) qv[s] = tb_ld(rs, (int)((((long)s * 64 + er) * H + en) * 4));
        const float dext = dpin_h + (((qv[0] + qv[1]) + qv[2]) + qv[3]);
        tb_cell_bwd(c2, dext, dhz2, dc2, rr2, d);
        float* const dg = a.dG2 + (tb + er) * K4 + en;
#pragma unroll
        for (int q = 0; q < 4; ++q) dg[q * H] = d[q];
      }
      // bf16 exchange row: the 4 units of (row er, gate q) are 4 adjacent tb_kperm positions (the
      // quad of lanes of row er shares erow, so the shuffles stay inside active quads)
      const int src = lane & ~3;
      float v[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[q][e] = __shfl(d[q], src + e, 64);
      if (erow && eu == 0) {
        const int p0 = tb_kperm(4 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          tp_st8(a.G2X, (int)(((long)par * 64 * K4 + tp_afl(er, p0 + 64 * q, K4)) * 2),
                 tp_u2{tp_pack(v[q][0], v[q][1]), tp_pack(v[q][2], v[q][3])});
      }
    }
    tp_publish(a, TB_PH_G2, tag);
    TB_STAMP(9);
    // ================= PROD2: [d h1 | d hz2_{t-1}] partial of (kb, nb)
    auto product = [&](const __bf16* X, const tp_bf8 (&wf)[2][8], float* out, int ph) {
      if (!tb_poll(a, ph, 16, tag, [&](int l) { return 16 * kb + l; })) sfail[0] = 1;
      const auto rs = tp_rsrc(X + (long)par * 64 * K4);
      const int vo = ((lane & 15) * 32 + 8 * (lane >> 4)) * 2;
      tp_f4 acc[2][4] = {};
#pragma unroll
      for (int h = 0; h < 4; ++h) {  // four batches of 2 k-steps, every load of a batch in flight
        tp_bf8 af[8];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) af[4 * i + mt] = tp_ldx4<true>(rs, vo, (mt * (K4 >> 5) + 8 * kb + 2 * h + i) * 1024);
        tp_wait(af);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
              acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[4 * i + mt], wf[nt][2 * h + i], acc[nt][mt], 0, 0, 0);
      }
      float* const ob = out + ((long)par * TB_NKB + kb) * 64 * TB_NOUT;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int m = 128 * nb + 32 * w + 16 * nt + jl;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) tb_st(ob, (int)(((16 * mt + 4 * g4 + i) * TB_NOUT + m) * 4), acc[nt][mt][i]);
      }
    };
    product(a.G2X, w2f, a.P2X, TB_PH_G2);
    __syncthreads();
    if (sfail[0]) return;
    tp_publish(a, TB_PH_P2, tag);
    TB_STAMP(10);
    // ================= CELL1: d h1 = Σ_kb P2 of the own N-block; d hz1 from step t+1's product 1
    TbCell c1{};
    float unused = 0.f;
    cell_load(0, c1, unused);
    float dh1 = 0.f, dhz1 = 0.f;
    if (!first) {
      if (!tb_poll(a, TB_PH_P1, TB_NKB, tagn, [&](int l) { return 16 * l + 8 + (g >> 5); })) sfail[0] = 1;
      if (erow) {
        const auto rs = tp_rsrc(a.P1X + (long)parn * TB_NKB * 64 * TB_NOUT);
        float pv[TB_NKB];
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) pv[k] = tb_ld(rs, (int)((((long)k * 64 + er) * TB_NOUT + H + en) * 4));
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) dhz1 += pv[k];
      }
      dhz1 += rr1;
    }
    if (!tb_poll(a, TB_PH_P2, TB_NKB, tag, [&](int l) { return 16 * l + (g >> 5); })) sfail[0] = 1;
    if (erow) {
      const auto rs = tp_rsrc(a.P2X + (long)par * TB_NKB * 64 * TB_NOUT);
      float pv[TB_NKB];
#pragma unroll
      for (int k = 0; k < TB_NKB; ++k) pv[k] = tb_ld(rs, (int)((((long)k * 64 + er) * TB_NOUT + en) * 4));
#pragma unroll
      for (int k = 0; k < TB_NKB; ++k) dh1 += pv[k];
    }
    __syncthreads();
    TB_STAMP(11);
    if (sfail[0]) return;
    {
      float d[4] = {0.f, 0.f, 0.f, 0.f};
      if (erow) {
        tb_cell_bwd(c1, dh1, dhz1, dc1, rr1, d);
        float* const dg = a.dG1 + (tb + er) * K4 + en;
#pragma unroll
        for (int q = 0; q < 4; ++q) dg[q * H] = d[q];
      }
      const int src = lane & ~3;
      float v[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[q][e] = __shfl(d[q], src + e, 64);
      if (erow && eu == 0) {
        const int p0 = tb_kperm(4 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          tp_st8(a.G1X, (int)(((long)par * 64 * K4 + tp_afl(er, p0 + 64 * q, K4)) * 2),
                 tp_u2{tp_pack(v[q][0], v[q][1]), tp_pack(v[q][2], v[q][3])});
      }
    }
    tp_publish(a, TB_PH_G1, tag);
    TB_STAMP(12);
    // ================= PROD1: [d ctx_{t-1} | d hz1_{t-1}] partial of (kb, nb)
    product(a.G1X, w1f, a.P1X, TB_PH_G1);
    __syncthreads();
    if (sfail[0]) return;
    tp_publish(a, TB_PH_P1, tag);
    TB_STAMP(13);
  }
#undef TB_STAMP
  // ---- the attention role's sums over the steps
  if (arow) {
#pragma unroll
    for (int r = 0; r < TB_PTW; ++r) {
      const int j = 16 * (w + 4 * r) + jl;
      if (j < Tin)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const tp_f4 v = {tp_aget(dkey[r][4 * mt]), tp_aget(dkey[r][4 * mt + 1]), tp_aget(dkey[r][4 * mt + 2]),
                           tp_aget(dkey[r][4 * mt + 3])};
          *reinterpret_cast<tp_f4*>(a.DKEYS + ((long)rb * Tin + j) * A + 32 * sq + 16 * mt + 4 * g4) = v;
        }
    }
    if (tid < 32) {
      a.dV[(long)rb * a.NT * A + 32 * sq + tid] = dva;
      a.dBA[(long)rb * a.NT * A + 32 * sq + tid] = dba;
    }
    {  // G^T tile of wave w: dims 16 (w >> 1) + 4 g4 + i, tap 16 (w & 1) + jl
      const int mt = w >> 1, nt = w & 1;
      float* const gs = a.DWGP + (long)rb * a.NT * 32 * A;
#pragma unroll
      for (int i = 0; i < 4; ++i) gs[(16 * nt + jl) * A + 32 * sq + 16 * mt + 4 * g4 + i] = gacc[i];
    }
  }
  if (g == 0 && tid == 0) a.ctl[1] = T;
}

__global__ __launch_bounds__(256) void k_tb_loc_grads(const float* __restrict__ G, const float* __restrict__ Wl, int F,
                                                      int A, int KW, float* __restrict__ dKc, float* __restrict__ dbc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (row < KW: tap, KW: bias) x filter
  if (i >= (KW + 1) * F) return;
  const int r = i / F, c = i % F;
  const float* gr = G + (long)(r < KW ? r : 31) * A;
  float v = 0.f;
  for (int k = 0; k < A; ++k) v += gr[k] * Wl[(long)c * A + k];
  if (r < KW)
    dKc[(long)r * F + c] = v;
  else
    dbc[c] = v;
}

void tb_loc_grads(const float* G, const float* Wl, int F, int A, int KW, float* dKc, float* dbc, hipStream_t s) {
  hipLaunchKernelGGL(k_tb_loc_grads, dim3(((KW + 1) * F + 255) / 256), dim3(256), 0, s, G, Wl, F, A, KW, dKc, dbc);
  TT2_HIP(hipGetLastError());
}

bool tb_device_ok(int dev) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
  if (prop.multiProcessorCount < TP_NB) return false;
  const void* k = reinterpret_cast<const void*>(k_tr_bwd_persist);
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tb_lds_bytes()) != hipSuccess)
    return false;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tr_bwd_persist, TP_NT, tb_lds_bytes()) != hipSuccess)
    return false;
  return nb >= 1;
}

// Cooperative launch: all TP_NB work-groups resident at once (or the launch fails); the spins rely on it.
void tb_launch(const TbArgs& a, hipStream_t s) {
  TbArgs arg = a;
  void* params[] = {&arg};
  TT2_HIP(launch_persistent(reinterpret_cast<const void*>(k_tr_bwd_persist), dim3(TP_NB), dim3(TP_NT), params,
                            (unsigned)tb_lds_bytes(), s));
}

}  // namespace tt2
