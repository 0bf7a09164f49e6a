// Persistent BPTT backward of the teacher-forced decoder in the training step (configs[4]; VERDICT
// r05 item 2): the reverse walk over the decoder steps that train.hip otherwise runs as four launches
// per step (k_tr_att_bwd_q + k_tr_fused<TF_BWD_H / TF_BWD_S / TF_PLAIN>) as ONE cooperative launch of
// 256 work-groups with the bf16 LSTM weights, the row's bf16 values quarter and the query columns
// resident on chip (helpers.py:62-133 and Architecture_wrappers.py:197-267 differentiated; the
// gradients tacotron.py:1194-1225 feeds to the optimizer).  It writes exactly what the per-step loop
// leaves for the weight-gradient products after the loop: dG1 / dG2 [T][B][4H], DQ [T][B][A],
// DCTX [T][B][D], DKEYS, the d v_a / d b_a partials and the d W_loc accumulators (DWGP); the prenet
// columns of d X1 come from one product after the launch.
#pragma once
#include <cstdint>

#include "train_persist.h"

namespace tt2 {

constexpr int TB_NKB = 16;  // K-blocks of the gate columns: units [64 kb, 64 kb + 64) x 4 gates
constexpr int TB_NNB = 16;  // N-blocks of the 2048 outputs of each backward product (128 each)
constexpr int TB_NPH = 5;   // flag phases (P1, Q, G2, P2, G1)
constexpr int TB_NOUT = 2 * TP_H;  // outputs of each product: [d h1 | d hz2] and [d ctx | d hz1]
constexpr int TB_TMAX = 160;       // encoder positions: the row's bf16 values quarter lives in LDS (80 KB)

struct TbArgs {
  int B, T, Tin, NT;         // NT: the per-row slot stride of dV / dBA / DWGP (train.hip's j-tiles)
  float z;                   // zoneout rate (only without keep masks)
  const __bf16* K1T;         // [4H][LX1] bf16 W1^T (hK1T)
  const __bf16* K2T;         // [4H][2H]  bf16 W2^T (hK2T)
  const __bf16* Wq;          // [H][A]    bf16 query_layer kernel (hWq)
  const float* va;           // [A]
  const float* KWT;          // [A][32] (tp_prepare): [a][tap] = (Kc·W_loc)[tap][a] for tap < KW
  const __bf16* values16;    // [B][Tin][D] bf16
  const int* lens;           // [B]
  const float* BPK;          // [T][TP_NB][4][TP_NT][4] the unit operands the persistent forward packed (TpArgs::BPK)
  // forward slots (train.hip layout)
  const float *ALN, *CUM, *TH;
  const float* dPIN;         // [T][B][H + D] d [h2 | ctx] from the frame / stop projections
  // outputs
  float *dG1, *dG2;          // [T][B][4H]
  __bf16 *DGT1, *DGT2;       // or null: bf16(dG)^T [4H][dgt_ld] (column t·64 + row; B = 64), the B^T operand the
                             // weight-gradient GEMMs stage (gemm_bf16_kc bt_pre), written beside the fp32 slots
  long dgt_ld;
  __bf16* DGR1;              // or null (with DGT1): bf16(dG1) row-major [T·64][4H], the A operand of the d X1 product
  float *DQ, *DCTX;          // [T][B][A], [T][B][D]
  float* DKEYS;              // [B][Tin][A]
  float *dV, *dBA;           // [B][NT][A]: slot b·NT holds row b's sums over steps and positions
  float* DWGP;               // [B][NT][32][A]: slot b·NT, G[tap][a] = Σ_t,j cum_t[j + tap - 15]·du[j][a]
  // exchange buffers
  __bf16 *G1X, *G2X;         // [2 parities][64 x 4H] bf16 A-fragment layout in the tb_kperm column order
  float *P1X, *P2X;          // per-K-block product partials, 2 parities of 16 MB: the d ctx block of P1
                             // (N-blocks < 8) row-major [kb][64][1024] in the first half (its reader takes
                             // one row), every unit-consumed block unit-major [nb][32][kb][64][4] (tb_uoff)
  __bf16* DQX;               // [2][64 x A] d query rows (bf16 A-fragment layout, K = A): each (row, quarter)
                             // writes its 32 dims, the unit role forms d h2 = dq·Wq^T
  __bf16* W1F;               // [TP_NB][4 waves][16 fragments][64 lanes][8] the W1 blocks, fragment-major
                             // (written at the start of the launch, streamed from L2 by each step's d X1
                             // product: one resident weight block per work-group fits the registers)
  unsigned long long* EX;    // [2][64][4][TP_TMAX] data-tagged d align partials
  unsigned* flags;           // [TB_NPH][TP_NREP][TP_NB] step tags (zeroed before the launch)
  int* ctl;                  // [0] = 1 + phase of a timed-out wait, [1] = steps completed
  long long* stamps;         // [TP_NB][32] s_memrealtime stage stamps of step stamp_step (diagnostic) or null
  int stamp_step;
};

// exchange column order of the dG rows: gate column q·H + u -> K-block u / 64 holds its 4 gates x 64
// units contiguously, so one product work-group reads one contiguous K range
__host__ __device__ inline int tb_kperm(int c) {
  const int q = c / TP_H, u = c % TP_H;
  return (u >> 6) * 256 + q * 64 + (u & 63);
}

size_t tb_lds_bytes();
bool tb_device_ok(int dev);
void tb_launch(const TbArgs& a, hipStream_t s);
// d Kc / d bc from the summed d W_loc accumulators G [32][A] (row 31 = Σ du = d b_a):
// dKc[tap][c] = Σ_a G[tap][a]·W_loc[c][a], dbc[c] = Σ_a G[31][a]·W_loc[c][a]
void tb_loc_grads(const float* G, const float* Wl, int F, int A, int KW, float* dKc, float* dbc, hipStream_t s);

}  // namespace tt2
