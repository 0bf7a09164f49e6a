// Wide-channel WaveNet generator (residual channels R = 128 / 256): the fork default
// (hparams.py:222-239: R=128, G=256, S=128, 20 layers / 2 stacks, Gaussian head) and the paper
// default (paper_hparams.py:199-204: R=256, G=512, S=256, 24 layers / 4 stacks, MoL head).
#pragma once
#include "common.h"

namespace tt2 {

constexpr int WW_THREADS = 256;  // 4 waves, one per SIMD: up to 512 registers per lane
constexpr int WW_TAPK = 32;      // tap rows (of [x(t-2d) | x(t-d)]) per k-slice
constexpr int WW_XK = 16;        // x(t) rows per k-slice
constexpr int WW_CK = WW_TAPK + WW_XK;
constexpr int WW_SOK = 16;       // z rows per skip/out k-slice

// CUs (work-groups) per layer: every layer's weights stay register-resident, 256 floats per lane
__host__ __device__ constexpr int ww_nc(int R) { return R == 128 ? 2 : 8; }

struct WideArgs {
  int T, L, per;              // samples, layers, layers per stack
  int b, Bg;                  // this launch's utterance, global batch (noise / cond indexing)
  const float* first_w; const float* first_b;  // [R], [R]
  const f32x4* conv_w;        // [L][NC][WW_CK][256] float4 (ww_pack_conv)
  const float* conv_b;        // [L][G] gate-permuted (gate_col order)
  const float* cond;          // [Bg][T][L][G] gate-permuted, cin_conv bias included
  const f32x4* so_w;          // [L][NC][WW_SOK][256] float4 (ww_pack_so)
  const float* so_b;          // [L][S + R] = [bs | bo]
  const float* f1_w; const float* f1_b;  // [S][S], [S]
  const float* f2_w; const float* f2_b;  // [S][C], [C]
  int C, legacy, res_legacy;
  float log_scale_min, log_scale_min_gauss;
  const float* u_mix; const float* u_log;  // [T][Bg][nr], [T][Bg] or null
  uint64_t seed;
  const float* teacher;       // [Bg][T] or null
  float* wav; int* kout; float* logits;    // [Bg][T], [Bg][T], [Bg][T][C]
  float* rings;               // per (layer, CU): [2d+1][R] fast-WaveNet queue, zeroed by the kernel
  unsigned long long* gran;   // [L][NC][S+R] + 1 sample granule; zeroed before the launch
  int* status;
  // R = 256 one-hop form (k_generate_wide<256, ·, true>, ww1_pack): per (layer, WG) [taps 32 | x rows 16
  // | z rows (rs·W_x·O of the previous layer) 16 | [out | skip] columns of the previous layer 16]
  // float4 per thread, for layers 0..L (L = the tail: the last layer's skips); gate biases with the
  // previous layer's out bias folded in [L][G] (gate-permuted)
  const f32x4* w1;
  const float* gb1;
  // layer 0 folded into the head (null: layer 0 runs on its own work-groups).  Layer 0's input is
  // the affine x_0(s) = y_{s-1}·fw + fb of the scalar sample, so each of its gate columns is
  // g + cond + Σ_k [tap k live] (y·U_k + V_k), U_k = W_k·fw, V_k = W_k·fb (k: x(s-2), x(s-1), x(s)).
  // Per z channel j: [a column | b column] x {U_0, U_1, U_2, g, V_0, V_1, V_2, 0}, float64-formed
  const float* l0;
};
constexpr int W1_NW = 80;         // float4 weights per thread and (layer, WG) in the one-hop form
constexpr int W1_GB = 3 * 256;    // granules per layer block: [z | x | skip]
bool ww_onehop(int R);            // R == 256 and TT2_WW_ONEHOP != 0
// one-hop packing of layer l (0..L; l == L the tail) for WG c: conv_l [3R][G] (null for the tail),
// out / skip kernels of layer l-1 (null for l == 0), M = rs·W_x(l)·O(l-1) [R z][G] (null for l == 0)
void ww1_pack(const float* conv_l, const float* out_prev, const float* skip_prev, const double* M, float rs, int c,
              std::vector<float>& out);

// Host packing of one layer's weights for CU c (row-major TF kernels: conv [3R][G], skip [R][S],
// out [R][R]); appended to out.
void ww_pack_conv(const float* conv, int R, int c, std::vector<float>& out);
void ww_pack_so(const float* skip, const float* outk, int R, int c, std::vector<float>& out);
size_t ww_ring_floats(int R, int L, int per);
size_t ww_lds_bytes(int R, int C);
int ww_blocks(int R, int L);
const void* ww_kernel(int R, bool gauss);

}  // namespace tt2
