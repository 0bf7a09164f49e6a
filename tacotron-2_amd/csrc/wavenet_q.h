// WaveNet synthesis for input_type 'mulaw-quantize' (one-hot input of Q classes, softmax head sampled
// by tf.multinomial; wavenet.py:433-452, 724-911) -- wavenet_q.hip.  One work-group per utterance.
#pragma once
#include <cstdint>

#include "common.h"

namespace tt2 {

constexpr int WQ_THREADS = 1024;
constexpr int WQ_QMAX = 1024;  // classes (one thread each in the sampler)

struct QGenArgs {
  int T, L, per, R, G, S, Q, Bg, legacy, res_legacy, k0;
  const float* first_w;  // [Q][R]: the input conv of a one-hot row is that row
  const float* first_b;  // [R]
  const float* conv_w;   // [L][3R][G] dilated conv, taps oldest first ([x(t-2d) | x(t-d) | x(t)] rows)
  const float* conv_b;   // [L][G]
  const float* cond;     // [Bg][T][L][G] conv1x1c (+ conv1x1g) terms incl. biases, or null (unconditional)
  const float* so_w;     // [L][R][S + R]: [skip | out] 1x1 kernels
  const float* so_b;     // [L][S + R]
  const float* f1_w; const float* f1_b;  // [S][S], [S]
  const float* f2_w; const float* f2_b;  // [S][Q], [Q]
  const float* u;        // [T][Bg] uniforms of the sampler, or null (device RNG keyed by seed)
  uint64_t seed;
  const float* teacher;  // [Bg][T] class indices (test_inputs, wavenet.py:752-759, 876-878) or null
  float* wav;            // [Bg][T] inv_mulaw_quantize of the drawn class
  int* kout;             // [Bg][T] drawn class (nullable)
  float* logits;         // [Bg][T][Q] (nullable)
  float* rings;          // [Bg][ring_floats] fast-WaveNet queues, zeroed before the launch
  long ring_floats;
};

// ring floats per utterance: Σ_l (2 d_l + 1) R
long wq_ring_floats(int R, int L, int per);
size_t wq_lds_bytes(int R, int G, int S, int Q);
void wq_launch(const QGenArgs& a, hipStream_t s);

}  // namespace tt2
