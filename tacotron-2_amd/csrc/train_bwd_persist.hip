// Persistent BPTT backward of the teacher-forced decoder (train_bwd_persist.h).
//
// Why: the per-step backward of train.hip is four launches per decoder step (attention backward,
// LSTM-2 cell backward behind d query·Wq^T, [d h1 | d hz2] = dG2·W2^T + LSTM-1 cell backward, d X1 =
// dG1·W1^T): 49.5 us per step, the bf16 values and the LSTM weights re-streamed from the MALL every
// step.  Here one launch walks t = T-1 .. 0 with them resident.
//
// Roles of work-group g (all 256 have all three):
//   attention  row rb = g & 63, quarter s = g >> 6: context channels [256 s, 256 s + 256) (the bf16
//              values quarter as MFMA A fragments in LDS, 80 KB at TB_TMAX = 160 positions) and
//              attention dims [32 s, 32 s + 32) (th, du, d keys, d query, the location-conv backward)
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
//        d query of the own dims (complete) -> DQ and the bf16 dq exchange rows DQX
//   CELL2  wait DQX of every (row, quarter), d h2 = d PIN + dq·Wq[own units]^T (one MFMA chain per
//        wave); d hz2 = Σ_kb P2_{t+1} + residual;
//        cell backward -> dG2 (fp32 slot + bf16 exchange)
//   PROD2  wait the K-block's 16 unit producers, dG2 block · W2 block -> P2
//   CELL1  wait P2 of the own N-block, d h1 = Σ_kb P2; d hz1 = Σ_kb P1_{t+1} + residual; cell
//        backward -> dG1
//   PROD1  wait the K-block's dG1, dG1 block · W1 block -> P1 (consumed at step t-1)
// Off the chain, after DQX is published: G[tap][a] += Σ_j cum_t[j + tap - 15]·du[j][a] (d W_loc, d Kc,
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
constexpr int TB_TM = TB_TMAX;           // encoder positions (capacity: the values quarter lives in LDS)
constexpr int TB_NPT = TB_TM / 16;       // position tiles
constexpr int TB_PTW = (TB_NPT + TB_NW - 1) / TB_NW;  // position tiles per wave (w + 4 r)
constexpr int TB_K4 = 4 * TP_H;          // gate columns
constexpr long TB_PSTRIDE = (long)TB_NNB * 32 * TB_NKB * 64 * 4;  // floats per parity of P1X / P2X
static_assert(TB_TM % 16 == 0 && TB_TM <= TP_TMAX && TP_NT == 256 && TP_A == 128 && TP_D == 1024 && TP_H == 1024,
              "train_bwd_persist geometry");

// LDS layout (floats).  The attention phase's du / M tiles and the products' staging share one
// region (different phases of a step, separated by barriers).
constexpr int TB_DUS = 34;                      // row stride of du (the G operand's column reads: 2 banks apart
                                                // per 8 positions, conflict-free per half wave)
constexpr int TB_OS = 132;                      // row stride of the staged product outputs
constexpr int TBL_DCH = 0;                      // [512] bf16: split halves of d ctx, hi [0, 256) | lo [256, 512)
constexpr int TBL_EP = TBL_DCH + 256;           // [TM] own d align partial
constexpr int TBL_DA = TBL_EP + TB_TM;          // [TM] d align, then de
constexpr int TBL_DS = TBL_DA + TB_TM;          // [TM] running d cum partial of the own dims
constexpr int TBL_CUM = TBL_DS + TB_TM;         // [TM + 64] cum_t at +15, zero padded
constexpr int TBL_RED = TBL_CUM + TB_TM + 64;   // [2][TB_NW][32] wave partials of dq / d v_a
constexpr int TBL_SC = TBL_RED + 2 * TB_NW * 32;  // [32] flags (ints)
constexpr int TBL_AL = TBL_SC + 32;             // [TM] the step's alignments a_j
constexpr int TBL_PA = TBL_AL + TB_TM;          // [TM] a_j · d a_j (the softmax backward's sum)
constexpr int TBL_CELL = TBL_PA + TB_TM;        // [17][256] the unit role's cell operands of the step
constexpr int TBL_DU = TBL_CELL + 17 * 256;     // [TM][34] du of the own dims (kept to the end of the step)
constexpr int TBL_U = TBL_DU + TB_TM * TB_DUS;  // union: M [TM][33] / PROD {A 32 KB, then out [64][132]}
constexpr int TBL_U_SZ = ((TB_TM + 32) * 33 > 64 * TB_OS) ? (TB_TM + 32) * 33 : 64 * TB_OS;
constexpr int TBL_VAL = TBL_U + TBL_U_SZ;       // [NPT tiles][8 k-steps][64 lanes] bf16 x 8: the values quarter
constexpr int TBL_END = TBL_VAL + TB_NPT * 8 * 64 * 4;
static_assert(TBL_U % 4 == 0 && TBL_VAL % 4 == 0 && TBL_DCH % 4 == 0 && 64 * TB_OS >= 8192,
              "16-byte aligned LDS regions; the product staging fits the union");

size_t tb_lds_bytes() { return sizeof(float) * (size_t)TBL_END; }

// work-group barrier for LDS hand-offs only: this wave's LDS operations complete, then s_barrier, WITHOUT
// the vmcnt(0) that __syncthreads()' release fence adds -- the HBM loads issued ahead (the next step's
// operands, the tanh tiles) stay in flight across it
__device__ __forceinline__ void tb_lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// sum over the 16 lanes of each lane row (xor within the low 4 lane bits; a butterfly reduce-scatter
// over 16 sums takes fewer shuffles but its selects cost the registers this kernel does not have)
__device__ __forceinline__ float tb_row16_sum(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float tb_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
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
// byte offset of (N-block nb, unit group m4 = 4-output group inside the block, K-block kb, row, e) in the
// unit-major partial layout [nb][m4][kb][row][4] (one parity): a unit work-group's 16 K-block partials of
// its 4 units are one contiguous 16 KB run
__device__ __forceinline__ int tb_uoff(int nb, int m4, int kb, int row, int e) {
  return ((((nb * 32 + m4) * TB_NKB + kb) * 64 + row) * 4 + e) * 4;
}
__device__ __forceinline__ float tb_ld(const __amdgpu_buffer_rsrc_t rs, int byte_off) {  // sc1 dword load
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, byte_off, 0, 16));
}
// the 4 gate gradients of (row er, unit en) at step t into bf16(dG)^T [4H][ld], column t·64 + er: a wave's
// store per gate writes 4 units x 16 consecutive rows (the work-group's 4 waves complete 128-byte runs)
__device__ __forceinline__ void tb_dgt(__bf16* DGT, long ld, int t, int er, int en, const float (&d)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long col = (long)q * TP_H + en;
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (__bf16)d[q]), tp_rsrc(DGT),
                                          (int)((col * ld + (long)t * 64 + er) * 2), 0, 0);
  }
}
// plain dword load of a read-only slot: wave-uniform base + per-lane byte offset (buffer addressing
// keeps the step loop free of per-lane 64-bit addresses, as train_persist.hip)
__device__ __forceinline__ float tb_lg(const float* base, int byte_off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(tp_rsrc(base), byte_off, 0, 0));
}

// LSTM cell backward of one (row, unit) (k_tr_lstm_bwd / tf_cell_bwd): the 4 gate gradients, the
// carried d(zoned c) updated, the zoneout residual (1 - kh)·dhz returned in res.  Operands: activated
// gates i j f o, c_new, c_prev (zoned), keep bits kc / kh (or 1 - z)
__device__ __forceinline__ void tb_cell_bwd(const float (&v)[8], float dext, float dhz, float& dc, float& res,
                                            float (&d)[4]) {
  const float si = v[0], tj = v[1], sf = v[2], so = v[3], cn = v[4], cp = v[5], kc = v[6], kh = v[7];
  const float dhn = dext + kh * dhz;
  const float tc = tanhf(cn);
  const float dcn = kc * dc + dhn * so * (1.f - tc * tc);
  const float dso = dhn * tc, dsf = dcn * cp, dsi = dcn * tj, dtj = dcn * si;
  d[0] = dsi * si * (1.f - si);
  d[1] = dtj * (1.f - tj * tj);
  d[2] = dsf * sf * (1.f - sf);
  d[3] = dso * so * (1.f - so);
  dc = (1.f - kc) * dc + dcn * sf;
  res = (1.f - kh) * dhz;
}

__global__ __launch_bounds__(TP_NT, 1) void k_tr_bwd_persist(TbArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __bf16* const dch = reinterpret_cast<__bf16*>(sm + TBL_DCH);  // [0, 256) hi, [256, 512) lo
  float* const ep = sm + TBL_EP;
  float* const da_s = sm + TBL_DA;
  float* const ds = sm + TBL_DS;
  float* const cum_s = sm + TBL_CUM;
  float* const red = sm + TBL_RED;
  float* const al_s = sm + TBL_AL;
  float* const pa_s = sm + TBL_PA;
  int* const sfail = reinterpret_cast<int*>(sm + TBL_SC + 16);
  float* const cel = sm + TBL_CELL;
  float* const dus = sm + TBL_DU;                    // ATT phase .. end of the step
  float* const ms = sm + TBL_U + 16 * 33;            // end of the step: M rows, 16 zero rows either side
  float* const stA = sm + TBL_U;                     // PROD phase: 32 A blocks of 1 KB
  float* const stO = sm + TBL_U;                     // PROD phase, after the products: [64][TB_OS] outputs
  tp_bf8* const valf = reinterpret_cast<tp_bf8*>(sm + TBL_VAL);
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
  // W2's block stays in registers; W1's goes to the fragment-major copy W1F that the d X1 product
  // streams from L2 every step (2 x 64 regs of resident weights do not fit beside the values quarter)
  tp_bf8 w2f[2][8];
  tp_bf8* const w1g = reinterpret_cast<tp_bf8*>(a.W1F) + ((long)g * TB_NW + w) * 16 * 64;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int m = 128 * nb + 32 * w + 16 * nt + jl;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int p0 = 32 * ks + 8 * g4;
      const int c0 = (p0 >> 6) * H + 64 * kb + (p0 & 63);
      tp_bf8 f1;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        w2f[nt][ks][e] = a.K2T[(long)(c0 + e) * 2 * H + m];  // W2[m][c]: m < H h1 rows, then hz2
        f1[e] = a.K1T[(long)(c0 + e) * LX1 + P + m];         // W1[P + m][c]: ctx rows, then hz1
      }
      w1g[(nt * 8 + ks) * 64 + lane] = f1;
    }
  }
  // ---- attention row constants
  // values quarter as A fragments in LDS (fragment-major, conflict-free reads): tile pt, k-step ks: lane
  // holds values16[rb][16 pt + jl][256 sq + 32 ks + 8 g4 .. + 8]
#pragma unroll
  for (int r = 0; r < TB_PTW; ++r) {
    const int pt = w + 4 * r;
    if (pt >= TB_NPT) break;  // wave-uniform
    const int j = 16 * pt + jl;
    const bool ok = arow && j < Tin;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      valf[(pt * 8 + ks) * 64 + lane] =
          ok ? *reinterpret_cast<const tp_bf8*>(a.values16 + ((long)rb * Tin + j) * D + 256 * sq + 32 * ks + 8 * g4) : tp_bf8{};
  }
  // the own 4 units' query rows as B fragments of the unit role's d h2 product (columns jl < 4 = units
  // 4g + jl, the others zero): k-step ks, lane holds Wq[4g + jl][32 ks + 8 g4 .. + 8]
  tp_bf8 wqb[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    wqb[ks] = jl < 4 ? *reinterpret_cast<const tp_bf8*>(a.Wq + (long)(4 * g + jl) * A + 32 * ks + 8 * g4) : tp_bf8{};
  // KW (the location conv folded through W_loc) as fp32 B fragments of the location-conv backward M = du·KW over
  // the own 32 dims (v_mfma_f32_16x16x4f32): tap tile nt, k-step k, lane holds KW[dim 32 sq + 4 k + g4][tap 16 nt + jl]
  // (tap 31, the bias column, zero)
  float kwf[2][8];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int tap = 16 * nt + jl;
      kwf[nt][k] = (arow && tap < 31) ? a.KWT[(32 * sq + 4 * k + g4) * 32 + tap] : 0.f;
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
  for (int e = tid; e < TM + 64; e += TP_NT) cum_s[e] = 0.f;
  for (int e = tid; e < TM; e += TP_NT) ds[e] = 0.f;
  if (tid == 0) sfail[0] = 0;

  // unit role: thread (row er, unit en); carried d c of both layers and the zoneout residuals
  const int er = tid >> 2, eu = tid & 3, en = 4 * g + eu;
  const bool erow = er < B;
  const int evo = er * H + en;
  float dc1 = 0.f, dc2 = 0.f, rr1 = 0.f, rr2 = 0.f;
  // The step's HBM operands (the unit role's cell operands of both layers, the attention row's align /
  // cum / d PIN ctx) are loaded one step AHEAD, at the start of the previous step's off-chain window
  // (LDS and MFMA work only, no global load waits there), and parked at the step's start: with vmcnt
  // in order, an HBM load issued in the step would hold every later poll and exchange load behind it
  // The cell operands come from the forward's packed copy (TpArgs::BPK: four coalesced 16-byte loads per
  // thread instead of 16 scattered dwords, 4x fewer bytes than the [T][B][4H] slots would fetch).
  tp_f4 cq[4];
  float cvd = 0.f, paj = 0.f, pcum = 0.f, pdctx = 0.f;
  auto prefetch = [&](int tt) {
    const long tbb = (long)tt * B;
    if (erow) {
      const auto rp = tp_rsrc(a.BPK + ((long)tt * TP_NB + g) * 4 * TP_NT * 4);
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
        cq[k4] = __builtin_bit_cast(tp_f4, __builtin_amdgcn_raw_buffer_load_b128(rp, (k4 * TP_NT + tid) * 16, 0, 0));
      cvd = tb_lg(a.dPIN + tbb * (H + D), (er * (H + D) + en) * 4);
    }
    if (arow) {
      const long rt = (tbb + rb) * Tin;
      const int tc = min(tid, Tin - 1);  // clamped: unconditional loads
      paj = tb_lg(a.ALN + rt, tc * 4);
      pcum = tb_lg(a.CUM + rt, tc * 4);
      pdctx = tb_lg(a.dPIN + (tbb + rb) * (H + D) + H + 256 * sq, tid * 4);
    }
  };
  prefetch(T - 1);
  __syncthreads();

  // product partial of (kb, nb): the K-block of dG (bf16 exchange rows X, parity par) staged in LDS in
  // one round trip (thread: 8 of its 32 one-KB (row tile, k-step) blocks; stored lane-major, each
  // fragment's 64 lanes contiguous, so the MFMA-side reads are conflict-free), then wave w's 2 x 4
  // tiles against its B fragments (resident, or streamed from the fragment-major copy wst in the same
  // round trip); the [64][128] fp32 partial staged in LDS and stored as 16-byte rows to
  // out[par][kb][row][128 nb ..)
  auto product = [&](const __bf16* X, const tp_bf8 (*wres)[8], const tp_bf8* wst, float* out, bool rowmajor, int ph,
                     int par, unsigned tag, long long* stp, int sb) {
    auto pst = [&](int i) {
      if (stp && tid == 0) stp[g * 32 + sb + i] = __builtin_amdgcn_s_memrealtime();
    };
    // the streamed weight fragments (independent of the step) go out before the wait on the dG block
    tp_bf8 ws[16];
    if (wst) {
      const auto rw = tp_rsrc(wst);
#pragma unroll
      for (int i = 0; i < 16; ++i) ws[i] = tp_ldx4<false>(rw, lane * 16, i * 1024);
    }
    if (!tb_poll(a, ph, 16, tag, [&](int l) { return 16 * kb + l; })) sfail[0] = 1;
    pst(0);
    {
      if (wst) tp_wait(ws);
      const auto rs = tp_rsrc(X + (long)par * 64 * K4);
      tp_bf8 f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {  // block b = w + 4 k: row tile b >> 3, k-step b & 7
        const int b = w + 4 * k;
        f[k] = tp_ldx4<true>(rs, lane * 16, ((b >> 3) * (K4 >> 5) + 8 * kb + (b & 7)) * 1024);
      }
      tp_wait(f);
      pst(1);
      // the 16-byte chunk at lane * 16 of a block is row lane >> 2, k-chunk lane & 3 = fragment lane
      // (lane >> 2) + 16 (lane & 3)
      const int dl = (lane >> 2) + 16 * (lane & 3);
#pragma unroll
      for (int k = 0; k < 8; ++k) *reinterpret_cast<tp_bf8*>(stA + (w + 4 * k) * 256 + dl * 4) = f[k];
    }
    __syncthreads();
    pst(2);
    tp_f4 acc[2][4] = {};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      tp_bf8 af[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) af[mt] = *reinterpret_cast<const tp_bf8*>(stA + (mt * 8 + ks) * 256 + lane * 4);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], wst ? ws[nt * 8 + ks] : wres[nt][ks], acc[nt][mt],
                                                                0, 0, 0);
    }
    __syncthreads();  // every wave's last A read before the outputs overwrite the staging area
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) stO[(16 * mt + 4 * g4 + i) * TB_OS + 32 * w + 16 * nt + jl] = acc[nt][mt][i];
    __syncthreads();
    pst(3);
    if (rowmajor) {  // d ctx block (nb < 8): [kb][row][1024]; store k: rows 8 k + (tid >> 5), 32 lanes per
                     // 512-byte row segment
      float* const ob = out + (long)par * TB_PSTRIDE + (long)kb * 64 * 1024;
      const int c4 = 4 * (tid & 31);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = 8 * k + (tid >> 5);
        tp_st16(ob, (r * 1024 + 128 * nb + c4) * 4, *reinterpret_cast<const tp_u4*>(stO + r * TB_OS + c4));
      }
    } else {  // unit-major [par][nb][m4][kb][row][4]: wave-instruction k = one 1-KB (m4, kb) run of 64 rows
      float* const ob = out + (long)par * TB_PSTRIDE;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int m4 = w + 4 * k;
        tp_st16(ob, ((((nb * 32 + m4) * TB_NKB + kb) * 64 + lane) * 4) * 4,
                *reinterpret_cast<const tp_u4*>(stO + lane * TB_OS + 4 * m4));
      }
    }
  };

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
    // ---- park the prefetched operands of step t (landed during the previous step's off-chain work):
    // the unit role's in LDS ([17][256], thread-private columns), the attention row's in registers
    // (slots 0-7 layer 2 (i j f o c_new c_prev kc kh), 8-15 layer 1, 16 d PIN (h part)); an attention row
    // parks behind its P1 poll, whose flag loads then travel beside the prefetch instead of after it
    auto park = [&] {
      if (erow) {
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
          for (int e = 0; e < 4; ++e) cel[(4 * k4 + e) * 256 + tid] = cq[k4][e];
        cel[16 * 256 + tid] = cvd;
      }
    };
    if (!arow) park();
    // ================= ATT
    if (arow) {
      const long rt = (tb + rb) * Tin;  // this row's [Tin] block of step t
      float aj = paj, cumv = pcum;
      // d ctx of channel 256 sq + tid = d PIN + Σ_kb P1_{t+1} (wave w: the N-block 2 sq + (w >> 1))
      float dctx = pdctx;
      // tanh of the own dims for the softmax / du stage, issued with the d align granules: the HBM latency
      // runs under the quarter exchange
      tp_f4 th[TB_PTW][2];
      auto load_th = [&] {
        const auto rth = tp_rsrc(a.TH + rt * A);
#pragma unroll
        for (int r = 0; r < TB_PTW; ++r) {
          const int j = min(16 * (w + 4 * r) + jl, Tin - 1);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
            th[r][mt] = __builtin_bit_cast(tp_f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rth, (j * A + 32 * sq + 16 * mt + 4 * g4) * 4, 0, 0));
        }
      };
      if (!first) {
        const int nbw = 2 * sq + (w >> 1);
        if (!tb_poll(a, TB_PH_P1, TB_NKB, tagn, [&](int l) { return 16 * l + nbw; })) sfail[0] = 1;
        TB_STAMP(1);
        const auto rs = tp_rsrc(a.P1X + (long)parn * TB_PSTRIDE);
        float pv[TB_NKB];
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) pv[k] = tb_ld(rs, ((k * 64 + rb) * 1024 + 256 * sq + tid) * 4);
        park();
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) dctx += pv[k];
      } else {
        park();
      }
      if (tid >= Tin) aj = cumv = 0.f;
      tp_bst(a.DCTX + (tb + rb) * D + 256 * sq, tid * 4, 0, dctx);
      {  // split-bf16 halves of d ctx: the B columns 0 (hi) and 1 (lo) of the d align product
        const __bf16 hi = (__bf16)dctx;
        dch[tid] = hi;
        dch[256 + tid] = (__bf16)(dctx - (float)hi);
      }
      if (tid < Tin) {
        cum_s[15 + tid] = cumv;
        al_s[tid] = aj;
      }
      tb_lds_bar();
      TB_STAMP(2);
      if (sfail[0]) return;
      // d align partial of the own channels: values quarter · (hi, lo) of d ctx on v_mfma_f32_16x16x32_bf16
      {
        tp_bf8 bfr[8];
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          const tp_bf8 v = *reinterpret_cast<const tp_bf8*>(dch + (jl == 1 ? 256 : 0) + 32 * ks + 8 * g4);
          bfr[ks] = jl < 2 ? v : tp_bf8{};
        }
        // the wave's position tiles interleaved k-step-major (each fragment read has the other tiles' MFMAs
        // to hide behind); a wave without a third tile recomputes the last one (identical values, and rows
        // past Tin are zero fragments: no branches)
        tp_f4 acc[TB_PTW];
#pragma unroll
        for (int r = 0; r < TB_PTW; ++r) acc[r] = tp_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
#pragma unroll
          for (int r = 0; r < TB_PTW; ++r) {
            const int pt = min(w + 4 * r, TB_NPT - 1);
            acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(valf[(pt * 8 + ks) * 64 + lane], bfr[ks], acc[r], 0, 0, 0);
          }
        // column 0 (hi) + column 1 (lo) of each row: DPP row_shl:1 brings lane jl + 1 to lane jl
#pragma unroll
        for (int r = 0; r < TB_PTW; ++r) {
          const int j0 = 16 * min(w + 4 * r, TB_NPT - 1) + 4 * g4;
          tp_f4 lo;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            lo[i] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc[r][i]), 0x101, 0xf, 0xf, false));
          if (jl == 0) {
            const tp_f4 d4 = *reinterpret_cast<const tp_f4*>(ds + j0);
            *reinterpret_cast<tp_f4*>(ep + j0) = acc[r] + lo + d4;
          }
        }
      }
      tb_lds_bar();
      // granules of the own partial, then the other quarters' (summed in quarter order)
      if (tid < Tin)
        __builtin_amdgcn_raw_buffer_store_b64(tp_u2{__float_as_uint(ep[tid]), tag},
                                              tp_rsrc(a.EX + (((long)par * 64 + rb) * 4 + sq) * TM), tid * 8, 0, 16);
      load_th();  // HBM latency under the quarter exchange
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
        if (act) {
          const float dv = ((e4[0] + e4[1]) + e4[2]) + e4[3];
          da_s[tid] = dv;
          pa_s[tid] = aj * dv;
        }
      }
      __syncthreads();
      TB_STAMP(4);
      if (sfail[0]) return;
      // softmax backward (attention.py:218): de_j = a_j (d a_j - Σ_k a_k d a_k), 0 past the length; every
      // wave forms the sum itself (same order in all: no barrier)
      float ssum;
      {
        float sp = 0.f;
#pragma unroll
        for (int k = 0; k < (TB_TM + 63) / 64; ++k) {
          const int j = lane + 64 * k;
          sp += j < Tin ? pa_s[j] : 0.f;
        }
        ssum = tb_wave_sum(sp);
      }
      // du of the own dims (energy-tile layout): d keys, d query, d v_a; du -> LDS
      float dqp[8], dvp[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) dqp[i] = dvp[i] = 0.f;
#pragma unroll
      for (int r = 0; r < TB_PTW; ++r) {
        const int pt = w + 4 * r;
        if (16 * pt >= Tin) break;  // wave-uniform
        const int j = 16 * pt + jl;
        const float dej = j < len ? al_s[j] * (da_s[j] - ssum) : 0.f;
        if (j >= Tin) th[r][0] = th[r][1] = tp_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          tp_f4 dv4;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float thv = th[r][mt][i];
            const float du = dej * vav[4 * mt + i] * (1.f - thv * thv);
            dkey[r][4 * mt + i] = tp_aput(tp_aget(dkey[r][4 * mt + i]) + du);
            dqp[4 * mt + i] += du;
            dvp[4 * mt + i] += dej * thv;
            dv4[i] = du;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) dus[j * TB_DUS + 16 * mt + 4 * g4 + i] = dv4[i];
        }
      }
      {  // the wave's sums over its positions of d query / d v_a per dim
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
      }
      __syncthreads();
      // wave 0: lanes < 32 sum the waves' d query / d v_a of dim lane; lanes < 4 pack the bf16 dq exchange row
      // (A-fragment layout, K = 128: the unit role forms d h2 = dq·Wq^T itself, bf16 operands as
      // k_tr_fused<TF_BWD_H>)
      float q = 0.f;
      if (w == 0) {
        float v = 0.f;
        const int dl = lane & 31;
#pragma unroll
        for (int ww = 0; ww < TB_NW; ++ww) {
          q += red[ww * 32 + dl];
          v += red[TB_NW * 32 + ww * 32 + dl];
        }
        if (lane < 32) {
          dba += q;
          dva += v;
        }
        float q8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) q8[e] = __shfl(q, 8 * (lane & 3) + e, 64);
        if (lane < 4) {
          const tp_u4 pk = {tp_pack(q8[0], q8[1]), tp_pack(q8[2], q8[3]), tp_pack(q8[4], q8[5]), tp_pack(q8[6], q8[7])};
          tp_st16(a.DQX, (int)(((long)par * 64 * A + tp_afl(rb, 32 * sq + 8 * lane, A)) * 2), pk);
        }
      }
      TB_STAMP(5);
      tp_publish(a, TB_PH_Q, tag);
      if (tid < 32) tp_bst(a.DQ + (tb + rb) * A + 32 * sq, tid * 4, 0, q);
      TB_STAMP(6);
    }
    // ================= CELL2: d hz2 from step t+1's product, d h2 from the dq rows of all quarters: both waits
    // first, then every load of the cell in one round trip
    if (!first && !tb_poll(a, TB_PH_P2, TB_NKB, tagn, [&](int l) { return 16 * l + 8 + (g >> 5); })) sfail[0] = 1;
    if (!tb_poll(a, TB_PH_Q, B, tag, [&](int l) { return 64 * w + l; })) sfail[0] = 1;  // wave w: quarter w
    __syncthreads();  // every quarter's poll behind this barrier; the parked operands visible
    TB_STAMP(8);
    if (sfail[0]) return;
    {
      // d h2 of (row, own unit) = dq[row]·Wq[unit]^T: wave w's row tile (rows 16 w ..) on one MFMA chain,
      // the 4 unit columns moved to the cell threads (row 16 w + (lane >> 2), unit lane & 3)
      // the P2_{t+1} partials of d hz2 go out with the dq rows: one round trip for both
      float dh2;
      float pv[TB_NKB];
      {
        const auto rq = tp_rsrc(a.DQX + (long)par * 64 * A);
        tp_bf8 af[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) af[ks] = tp_ldx4<true>(rq, ((lane & 15) * 32 + 8 * (lane >> 4)) * 2, (w * 4 + ks) * 1024);
        if (erow && !first) {
          const auto rp = tp_rsrc(a.P2X + (long)parn * TB_PSTRIDE);
#pragma unroll
          for (int k = 0; k < TB_NKB; ++k) pv[k] = tb_ld(rp, tb_uoff(8 + (g >> 5), g & 31, k, er, eu));
        }
        tp_wait(af);
        tp_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], wqb[ks], acc, 0, 0, 0);
        const int rl = lane >> 2, srcl = (lane & 3) + 16 * (rl >> 2);
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = __shfl(acc[i], srcl, 64);
        const int ri = rl & 3;
        dh2 = ri == 0 ? v[0] : ri == 1 ? v[1] : ri == 2 ? v[2] : v[3];
      }
      float d[4] = {0.f, 0.f, 0.f, 0.f};
      if (erow) {
        float c[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = cel[k * 256 + tid];
        float dhz2 = 0.f;
        if (!first) {
#pragma unroll
          for (int k = 0; k < TB_NKB; ++k) dhz2 += pv[k];
          dhz2 += rr2;
        }
        const float dext = cel[16 * 256 + tid] + dh2;
        tb_cell_bwd(c, dext, dhz2, dc2, rr2, d);
      }
      // bf16 exchange row: the 4 units of (row er, gate q) are 4 adjacent tb_kperm positions (the quad
      // of lanes of row er shares erow, so the shuffles stay inside active quads)
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
      tp_publish(a, TB_PH_G2, tag);
      // the fp32 dG2 slot (read after the launch) behind the publish: its scattered stores drain at the
      // next publish instead of holding this one
      if (erow) {
#pragma unroll
        for (int q = 0; q < 4; ++q) tp_bst(a.dG2 + tb * K4, (er * K4 + en + q * H) * 4, 0, d[q]);
        if (a.DGT2) tb_dgt(a.DGT2, a.dgt_ld, t, er, en, d);
      }
    }
    TB_STAMP(9);
    // ================= PROD2: [d h1 | d hz2_{t-1}] partial of (kb, nb)
    product(a.G2X, w2f, nullptr, a.P2X, false, TB_PH_G2, par, tag, stp, 14);
    __syncthreads();
    if (sfail[0]) return;
    tp_publish(a, TB_PH_P2, tag);
    TB_STAMP(10);
    // ================= CELL1: d h1 = Σ_kb P2 of the own N-block; d hz1 from step t+1's product 1
    if (!first && !tb_poll(a, TB_PH_P1, TB_NKB, tagn, [&](int l) { return 16 * l + 8 + (g >> 5); })) sfail[0] = 1;
    if (!tb_poll(a, TB_PH_P2, TB_NKB, tag, [&](int l) { return 16 * l + (g >> 5); })) sfail[0] = 1;
    __syncthreads();
    TB_STAMP(11);
    if (sfail[0]) return;
    {
      float d[4] = {0.f, 0.f, 0.f, 0.f};
      if (erow) {
        float pa[TB_NKB], pb[TB_NKB];
        const auto r1 = tp_rsrc(a.P1X + (long)parn * TB_PSTRIDE);
        const auto r2 = tp_rsrc(a.P2X + (long)par * TB_PSTRIDE);
        if (!first)
#pragma unroll
          for (int k = 0; k < TB_NKB; ++k) pa[k] = tb_ld(r1, tb_uoff(8 + (g >> 5), g & 31, k, er, eu));
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) pb[k] = tb_ld(r2, tb_uoff(g >> 5, g & 31, k, er, eu));
        if (stp && tid == 0) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          stp[g * 32 + 22] = __builtin_amdgcn_s_memrealtime();
        }
        float c[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = cel[(8 + k) * 256 + tid];
        float dh1 = 0.f, dhz1 = 0.f;
#pragma unroll
        for (int k = 0; k < TB_NKB; ++k) dh1 += pb[k];
        if (!first) {
#pragma unroll
          for (int k = 0; k < TB_NKB; ++k) dhz1 += pa[k];
          dhz1 += rr1;
        }
        tb_cell_bwd(c, dh1, dhz1, dc1, rr1, d);
        if (stp && tid == 0) stp[g * 32 + 23] = __builtin_amdgcn_s_memrealtime();
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
        if (a.DGR1)  // the same 4 units of gate q, row-major (off the chain: drained by a later publish)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            __builtin_amdgcn_raw_buffer_store_b64(tp_u2{tp_pack(v[q][0], v[q][1]), tp_pack(v[q][2], v[q][3])},
                                                  tp_rsrc(a.DGR1), (int)((((long)t * 64 + er) * K4 + q * H + 4 * g) * 2), 0, 0);
      }
      tp_publish(a, TB_PH_G1, tag);
      if (erow) {
#pragma unroll
        for (int q = 0; q < 4; ++q) tp_bst(a.dG1 + tb * K4, (er * K4 + en + q * H) * 4, 0, d[q]);
        if (a.DGT1) tb_dgt(a.DGT1, a.dgt_ld, t, er, en, d);
      }
    }
    TB_STAMP(12);
    // ================= PROD1: [d ctx_{t-1} | d hz1_{t-1}] partial of (kb, nb)
    product(a.G1X, w2f, w1g, a.P1X, nb < TB_NNB / 2, TB_PH_G1, par, tag, stp, 18);
    __syncthreads();
    if (sfail[0]) return;
    tp_publish(a, TB_PH_P1, tag);
    TB_STAMP(13);
    if (t > 0) prefetch(t - 1);
    TB_STAMP(24);
    if (arow) {
      // ---- off the chain: d W_loc accumulators and the location-conv backward of the own dims, both on
      // fp32 v_mfma_f32_16x16x4f32 (exact products, operands straight from LDS)
      {  // G^T[a][tap] += Σ_j du[j][a]·cum_t[j + tap - 15]: wave w -> dim tile w >> 1, tap tile w & 1; K = the
         // positions, 4 per MFMA (rows past Tin of du and cum are zero), 4 accumulation chains
        const int mt = w >> 1, nt = w & 1;
        const int nk16 = (Tin + 15) >> 4;
        tp_f4 gq[4] = {};
#pragma unroll
        for (int k16 = 0; k16 < TB_NPT; ++k16) {
          if (k16 >= nk16) break;  // wave-uniform
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int j = 16 * k16 + 4 * q + g4;
            gq[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(dus[j * TB_DUS + 16 * mt + jl], cum_s[j + 16 * nt + jl], gq[q],
                                                         0, 0, 0);
          }
        }
        gacc += (gq[0] + gq[1]) + (gq[2] + gq[3]);
      }
      TB_STAMP(25);
#pragma unroll
      for (int q6 = 0; q6 < 2 * TB_PTW; ++q6) {  // M tiles (position tile, tap tile) = w + 4 q6, K = the 32 own dims
        const int idx = w + 4 * q6, pt = idx >> 1, nt = idx & 1;
        if (16 * pt >= Tin) continue;  // wave-uniform
        tp_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dus[(16 * pt + jl) * TB_DUS + 4 * k + g4], kwf[nt][k], acc, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) ms[(16 * pt + 4 * g4 + i) * 33 + 16 * nt + jl] = acc[i];
      }
      {  // the zero pad rows of the diagonal sum (the product staging shares the region)
        const int r1 = 16 * ((Tin + 15) >> 4);
        for (int e = tid; e < 16 * 33; e += TP_NT) {
          ms[e - 16 * 33] = 0.f;
          ms[r1 * 33 + e] = 0.f;
        }
      }
      tb_lds_bar();
      TB_STAMP(26);
      if (tid < Tin) {  // d cum_t[i] += Σ_tap M[i - tap + 15][tap] (4 independent chains; rows -16.. and
                        // past the tiles are the zero pad, tap 31 the zero column: no conditions)
        float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 32; ++tap) v[tap & 3] += ms[(tid - tap + 15) * 33 + tap];
        ds[tid] += (v[0] + v[1]) + (v[2] + v[3]);
      }
    }
    TB_STAMP(7);
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
