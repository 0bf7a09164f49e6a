// fp32 MFMA GEMM with implicit-im2col loaders and fused epilogues (gfx950).
#pragma once
#include "common.h"

namespace tt2 {

enum AMode { A_DENSE = 0, A_CONV1D = 1, A_CONV2D = 2 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_BN_RELU = 9 };  // BN_RELU: BN then ReLU (modules.py:507-510)

struct GemmArgs {
  int M = 0, N = 0, K = 0;
  int a_mode = A_DENSE;
  const float* A = nullptr;
  long lda = 0;            // dense: row stride
  // conv1d ("same", stride 1): X[b][t][c] at X + b*xs_b + t*xs_t + c; m = b*T + t; k = tap*C + c
  int T = 0, C = 0, kw = 0, pad = 0;
  long xs_b = 0, xs_t = 0;
  // conv2d NHWC: X[n][h][w][c]; m = (n*Ho + ho)*Wo + wo; k = (i*kw2 + j)*C + c
  int H = 0, Wd = 0, Ho = 0, Wo = 0, kh = 0, kw2 = 0, sh = 1, sw = 1, pt = 0, pl = 0;
  const float* Bw = nullptr;  // [K][N] row-major
  long ldb = 0;
  float* Cout = nullptr;      // row-major [M][ldc]
  long ldc = 0;
  // epilogue: y = acc + bias; y = act(y); y = y*bn_scale + bn_shift; y += residual; clip
  const float* bias = nullptr;
  int act = ACT_NONE;
  const float* bn_scale = nullptr;
  const float* bn_shift = nullptr;
  const float* residual = nullptr;
  long ldr = 0;
  int clip = 0;
  float clip_lo = 0.f, clip_hi = 0.f;
  // arithmetic: 0 = fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products); 1 = split fp16x3:
  // every operand x = hi + lo (two fp16, after an exact power-of-two pre-scale A·2^4, B·2^10 that
  // keeps lo out of fp16 subnormals), A·B = Ah·Bh + Ah·Bl + Al·Bh on v_mfma_f32_32x32x16_f16 with
  // fp32 accumulation (the dropped lo·lo term is ~2^-22 relative; fp16 products are exact in
  // fp32) -- 3/16 of the fp32 MFMA cost, ~1e-7 relative error.  Needs |A| < 4e3, |B| < 64.
  // 2 = bf16 operands (round-to-nearest-even), fp32 accumulation: mixed-precision training.
  int split16 = 0;
  // split-K for skinny products (fp32 path): when kpart != nullptr the dispatcher may split K over
  // blockIdx.z so a 64-row GEMM fills the chip; raw partials go to kpart (>= kpart_floats floats,
  // caller-owned, stream-ordered) and one reduce launch applies the epilogue.
  float* kpart = nullptr;
  // split16 == 2 only: B given pre-transposed in bf16, Bt16[n * ldbt + k] (ldbt % 8 == 0, 16-byte
  // aligned) -- half the weight bytes and one 16-byte load per 8 k (training weights, converted
  // once per optimizer step).  Bw is ignored when set.
  const void* Bt16 = nullptr;
  long ldbt = 0;
  // split16 == 1: pre-split planes from split_weights() (Bt16 = hi, Bt16lo = lo, both [N][ldbt])
  const void* Bt16lo = nullptr;
  long kpart_floats = 0;
  int ksplit = 1;  // set by the dispatcher
  int raw = 0;     // internal: partials only (gemm_raw)
};

// Pre-split fp16 planes of a static weight for split16 == 1 (see GemmArgs::Bt16lo).
struct SplitB {
  DevBuf hi, lo;
  long ldbt = 0;
  void set(GemmArgs& g) const {
    if (hi.p) {
      g.Bt16 = hi.p;
      g.Bt16lo = lo.p;
      g.ldbt = ldbt;
    }
  }
};
void split_weights(const float* B, int K, int N, long ldb, SplitB& out, hipStream_t s);

// ---- conv1d 'same' over pre-split activation planes ---------------------------
// Activations between stacked conv layers live as two fp16 planes (hi, lo of x·2^4, the split
// GemmArgs::split16 == 1 applies at load) in a PADDED row layout: CX_G guard rows, then for every
// batch row b the CX_P zero rows, its T frames, CX_P zero rows (Tp = T + 2·CX_P rows per b), then
// guard rows up to the 256-row tile multiple + CX_G.  Channel stride Cp (C rounded up to 32, zero
// padded).  A conv tap is then a plain row shift, so the product streams dense 16-byte rows with no
// im2col arithmetic and no per-load split, and the producing layer writes the next layer's planes
// from its epilogue (pad rows as zeros).
constexpr int CX_P = 2, CX_G = 2, CX_BM = 128, CX_BN = 128;
inline long cx_rows(int B, int T) { return 2L * CX_G + (((long)B * (T + 2 * CX_P) + 255) / 256) * 256; }
struct ConvX3Args {
  const _Float16 *Ah = nullptr, *Al = nullptr;  // input planes (allocation base: guard rows first)
  int Cp = 0;                                   // input channel stride (multiple of 32)
  int B = 0, T = 0, kw = 1;                     // 'same' conv of width kw (odd, <= 2·CX_P + 1)
  const _Float16 *Bh = nullptr, *Bl = nullptr;  // weights [N][ldbt], k = tap·Cp + c (split_conv_weights)
  long ldbt = 0;
  int N = 0;
  const float *bias = nullptr, *bn_scale = nullptr, *bn_shift = nullptr;
  int act = ACT_NONE;
  _Float16 *Oh = nullptr, *Ol = nullptr;  // split output planes, channel stride N (N % 128 == 0), or
  float* Cout = nullptr;                  // fp32 output rows b·T + t (stride ldc) with residual / clip
  long ldc = 0;
  const float* residual = nullptr;
  long ldr = 0;
  int clip = 0;
  float clip_lo = 0.f, clip_hi = 0.f;
  // split-K for few-row products (the text encoder's 6.4k rows): ks > 1 slices K over blockIdx.y
  // of the 128 x 128 kernel, raw fp32 partials [ks][B·Tp][N] go to part (>= part_floats floats,
  // stream-ordered) and one reduce launch applies the epilogue and writes the output
  int ks = 1;
  float* part = nullptr;
  long part_floats = 0;
};
void conv_x3(const ConvX3Args& a, hipStream_t s);
// fp32 X[b][t][c] (batch stride xs_b, frame stride C) -> padded planes (zero pads, channels C..Cp)
void split_rows(const float* X, int B, int T, int C, long xs_b, _Float16* hi, _Float16* lo, int Cp, hipStream_t s);
// conv weight W[kw][C][N] fp32 -> pre-scaled split planes [N][kw·Cp] (zero for c >= C)
void split_conv_weights(const float* W, int kw, int C, int Cp, int N, SplitB& out, hipStream_t s);

// ---- large bf16 product C[M][N] = A[M][K]·B[K][N] (training weight / conv gradients) ----------
// A (K contiguous, row stride lda) and B (N contiguous, row stride ldb) are rounded to bf16 into
// padded K-contiguous copies a16 [Mp][Kp] and b16 [Np][Kp] (B transposed on the way), then a
// 256 x 256 x 64 LDS-DMA MFMA kernel (fp32 accumulation) with K split over work-groups when the
// tiles alone do not fill the chip (partials in part, one combine launch).  The buffers grow on
// demand; all work is ordered on stream s.
// a_kmajor: A is given as its transpose At[K][M] (row stride lda), e.g. the activations X[T·B][M] of
// a weight gradient X^T·dG, and is transposed by the same conversion pass as B.
// conv: A is the transposed im2col of a 'same' conv1d input X[b][t][c] (batch / frame strides xs_b,
// xs_t): A[tap·C + c][b·T + t] = X[b][t + tap - pad][c] (0 outside [0, T)), M = kw·C, K = B·T --
// the conv weight gradient im2colᵀ·dZ, gathered straight into the bf16 copy.
struct KcConvA {
  const float* x = nullptr;
  long xs_b = 0, xs_t = 0;
  int B = 0, T = 0, C = 0, kw = 0, pad = 0;
};
void gemm_bf16_kc(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C, long ldc,
                  DevBuf& a16, DevBuf& b16, DevBuf& part, hipStream_t s, bool a_kmajor = false,
                  const KcConvA* conv = nullptr, const __bf16* bt_pre = nullptr, const __bf16* a_pre = nullptr);
// the [Np][Kp] bf16 B^T layout gemm_bf16_kc stages (Np = N rounded to 256; Kp = K rounded to its k-step split),
// for producers that write it themselves (gemm_bf16_kc(..., bt_pre) skips the conversion pass)
void gemm_bf16_kc_bt_dims(int M, int N, int K, long* Np, long* Kp);

// gemm_bf16_kc's kernel as a 'same' conv1d over padded bf16 planes (one plane, the CX_* row layout
// above, channel stride Cp % 64 == 0): out[b·T + t][n] = act(Σ_k ... + bias[n]) for n < N, with the
// weights as Bt[Np][ldbt] bf16 (k = tap·Cp + c, Np >= N rounded up to 256 rows) -- the training
// Postnet's forward and input-gradient convolutions.
struct KcEpi {
  int T = 0, B = 0;  // T > 0: conv epilogue (padded rows -> frames)
  const float* bias = nullptr;
};
void conv_bf16_planes(const __bf16* planes, int Cp, int B, int T, int kw, const __bf16* Bt, long ldbt, int N,
                      const float* bias, int act, float* out, long ldo, hipStream_t s);
// B[K][N] fp32 -> out[Np][Kp] bf16 transposed, zero padded (Kp, Np multiples of 64)
void kc_transpose_bf16(const float* B, int K, int N, long ldb, __bf16* out, int Kp, int Np, hipStream_t s);

void gemm(const GemmArgs& a, hipStream_t s);
// Same product, but the raw fp32 partial sums are left in a.kpart as [ks][M][N] (no epilogue, no
// combine launch; ks >= 1 is returned) for a caller-fused combine.  a.kpart is required.
int gemm_raw(const GemmArgs& a, hipStream_t s);

}  // namespace tt2
