// Persistent teacher-forced decoder forward of the training step (configs[4]; VERDICT r03 item 4c /
// r04 item 2): the whole TacoTrainingHelper dynamic_decode loop (helpers.py:62-133 at ratio 1,
// Architecture_wrappers.py:197-267, tacotron.py:1002-1109's training graph) as ONE cooperative
// launch of 256 work-groups with the bf16 LSTM weights resident on chip.  It writes exactly the
// activation slots the per-step launch loop of train.hip writes (X1 / X2 / PIN / G / CN / C / TH /
// FALL / ALN / ALIGN / CUM), so the backward is unchanged.
#pragma once
#include <cstdint>

#include "common.h"

namespace tt2 {

constexpr int TP_NB = 256;    // work-groups: LSTM tile of 4 hidden units x 4 gates; attention (row, quarter)
constexpr int TP_NT = 256;    // 4 waves, one per SIMD: 512 registers per lane (VGPR + AGPR)
constexpr int TP_H = 1024;    // decoder_lstm_units
constexpr int TP_P = 256;     // prenet units
constexpr int TP_D = 1024;    // memory width (attention values / context)
constexpr int TP_A = 128;     // attention_dim
constexpr int TP_F = 32;      // attention_filters
constexpr int TP_TMAX = 192;  // encoder positions: the row's values quarter lives in VGPRs
constexpr int TP_KWMAX = 31;  // attention_kernel
constexpr int TP_NREP = 8;    // replicas of every flag line (32 pollers per line)
constexpr int TP_LX1 = TP_P + TP_D + TP_H;

struct TpArgs {
  int B, T, Tin, KW;
  float z;                   // zoneout rate (only without keep masks)
  const __bf16* K1T;         // [4H][LX1] bf16 W1^T (hK1T)
  const __bf16* K2T;         // [4H][2H]  bf16 W2^T (hK2T)
  const __bf16* Wq;          // [H][A]    bf16 query_layer kernel (hWq)
  const float* b1;           // [4H]
  const float* b2;           // [4H]
  const float* Kc;           // [KW][F] location conv kernel
  const float* bc;           // [F]
  const float* Wl;           // [F][A] location_features_layer
  const float* va;           // [A]
  const float* ba;           // [A]
  const float* KWT;          // [A][32]: [a][tap < KW] = (Kc·W_loc)[tap][a], [a][31] = (bc·W_loc)[a] (tp_prepare)
  const float* keys;         // [B][Tin][A] fp32
  const __bf16* values16;    // [B][Tin][D] bf16
  const int* lens;           // [B]
  const uint8_t* zm;         // [T][4][B][H] zoneout keep bits or null
  const __bf16* preh;        // [T][64 x P] prenet rows, bf16, A-fragment layout (tp_afl, K = P)
  // activation slots (train.hip layout)
  float *X1, *X2, *PIN, *G1, *G2, *CN1, *CN2, *C1, *C2, *ALIGN, *CUM, *TH, *FALL, *ALN;
  // exchange buffers, [2 parities][64 x K] bf16 in A-fragment layout; granules [2][64][4][TMAX]
  __bf16 *CX, *H1X, *Z1X, *H2X, *Z2X;
  unsigned long long* EX;
  // the persistent backward's unit operands, or null: [T][TP_NB][4][TP_NT][4] floats, thread (row er, unit 4g + eu)
  // of work-group g: [layer-2 i j f o | c_new c_prev kc kh | layer-1 i j f o | c_new c_prev kc kh] (activated
  // gates, the carried c before the step, the zoneout keep factors) -- one coalesced 16-byte store per quad
  float* BPK;
  long long* stamps;         // [TP_NB][32] s_memrealtime stage stamps of step stamp_step (diagnostic) or null
  int stamp_step;
  int oc_mode;               // placement of the off-chain products (TT2_TP_OC, A/B): see k_tr_persist
  unsigned* flags;           // [3 phases][TP_NREP][TP_NB] step tags (zeroed before the launch)
  int* ctl;                  // [0] = 1 + phase of a timed-out wait, [1] = steps completed
};

// A-fragment layout of a [64][K] bf16 operand for v_mfma_f32_16x16x32_bf16: 16-row tiles x 32-deep
// k-steps x [16 rows][32 k], so a wave's fragment of one (tile, k-step) is one contiguous kilobyte
__host__ __device__ inline long tp_afl(int r, int k, int K) {
  return ((long)((r >> 4) * (K >> 5) + (k >> 5)) * 16 + (r & 15)) * 32 + (k & 31);
}

size_t tp_lds_bytes();
bool tp_device_ok(int dev);
void tp_launch(const TpArgs& a, hipStream_t s);
// prenet rows X1[t][b][0:P] (fp32, row stride ld) -> bf16 A-fragment layout, rows >= B zero
void tp_prenet_rows(const float* X1, long ld, int B, int T, __bf16* preh, hipStream_t s);
// KWT (above) from the location conv kernel Kc [KW][F], its bias bc [F] and W_loc [F][A]
void tp_prepare(const float* Kc, const float* bc, const float* Wl, float* KWT, hipStream_t s);
// the location features of every step, FALL[t][b][j][c] = bc[c] + Σ_tap CUM[t][b][j + tap - 15]·Kc[tap][c]
// (the launch loop's tr_locf_tile order), from the cumulative alignments the persistent loop wrote
void tp_location_features(const float* CUM, const float* Kc, const float* bc, int B, int T, int Tin, float* FALL,
                          hipStream_t s);

}  // namespace tt2
