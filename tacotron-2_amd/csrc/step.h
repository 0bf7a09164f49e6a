// Single decoder step with explicit state in / state out (tt2_decoder_step): the parity seam for
// TacotronDecoderCell.__call__ (Architecture_wrappers.py:197-267).  Plain fp32 kernels over
// row-major weights (one thread per output, k in order): not a hot path -- tt2_decode runs the
// fused loop -- but the exact per-step semantics in a form a test can drive one call at a time.
#pragma once
#include "common.h"

namespace tt2 {

struct StepWeights {               // row-major device copies of the TF variables
  const float *pre_w1, *pre_b1;    // [nm][P], [P]
  const float *pre_w2, *pre_b2;    // [P][P], [P]
  const float *k1, *b1;            // [P + D + H][4H], [4H]   (gate order i, j, f, o)
  const float *k2, *b2;            // [2H][4H], [4H]
  const float *wq;                 // [H][A]
  const float *wconv;              // [KL][F] (location conv, 1 input channel; its bias is folded in keys)
  const float *wloc;               // [F][A]
  const float *va;                 // [A]
  const float *wf, *bf;            // [H + D][nm], [nm]
  const float *ws, *bs;            // [H + D][1], [1]
};

struct StepDims {
  int B, T, nm, P, H, D, A, F, KL;
  float zo;
  int cumulative, constraint, monotonic, win, mask_encoder, smoothing;
};

struct StepIO {
  const float* keys;      // [B][T][A] memory_layer(values) + b_a + b_conv·W_loc (tt2_encode)
  const float* values;    // [B][T][D]
  const int* lengths;     // [B]
  const float* frame_in;  // [B][nm]
  const uint8_t* masks;   // [2][B][P] prenet keep bits
  const float *h1, *c1, *h2, *c2, *ctx, *cum;  // state in
  const int* max_att;
  float *h1o, *c1o, *h2o, *c2o, *ctxo, *cumo;  // state out
  int* max_att_o;
  float *frame, *stop, *align;                 // [B][nm], [B], [B][T]
  float* scratch;         // step_scratch_floats(d)
};

size_t step_scratch_floats(const StepDims& d);
void decoder_step_launch(const StepWeights& w, const StepDims& d, const StepIO& io, hipStream_t s);

}  // namespace tt2
