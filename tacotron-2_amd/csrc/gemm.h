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
  // optional second output of the pre-residual value (unused = nullptr)
};

void gemm(const GemmArgs& a, hipStream_t s);

}  // namespace tt2
