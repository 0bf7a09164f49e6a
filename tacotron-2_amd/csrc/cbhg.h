// CBHG post-processing network + linear-spectrogram projection (modules.py:110-184; its caller is
// commented out in the reference, tacotron.py:466-478: linear_outputs = clip(FrameProjection(
// num_freq)(CBHG(mel_outputs, None)))).  Built when tt2_config.predict_linear is set.
#pragma once
#include "common.h"
#include "gemm.h"

namespace tt2 {

struct CbhgModel {
  bool on = false;
  int nm = 0, K = 0, C = 0, pool = 0, proj = 0, kp = 0, nhw = 0, Hu = 0, R = 0, nf = 0;
  int clip = 0;
  float clip_lo = 0.f, clip_hi = 0.f;
  DevBuf bank_w[16], bank_b[16], bank_s[16], bank_h[16];
  DevBuf p1_w, p1_b, p1_s, p1_h, p2_w, p2_b, p2_s, p2_h;
  DevBuf dn_w, dn_b;        // residual -> highway width (when num_mels != highway units)
  DevBuf hw_w[8], hw_b[8];  // [Hu][2Hu] = [W_H | W_T], [2Hu]
  DevBuf gx_w, gx_b, g_whg, g_whc;  // BiGRU: x rows [Hu][2·3R] (fw | bw), recurrent rows per direction
  DevBuf pj_w, pj_b;        // [2R][num_freq]
  DevBuf bank, pool_out, p1, hw[2], ht, xg, gru;  // activations, sized per call
};

// shapes + weights (TF names under prefix: "<prefix>CBHG_postnet/...",
// "<prefix>cbhg_linear_specs_projection/..."); bn(scope, C, scale, shift) uploads BN constants
void cbhg_load(CbhgModel& m, const WeightMap& wm, const std::string& prefix, int num_mels, int kernels,
               int conv_channels, int pool_size, int projection, int projection_kernel, int highway_layers,
               int highway_units, int rnn_units, int num_freq);
// mels [B][T][nm] (device) -> linear [B][T][num_freq] (device), on stream s
void cbhg_linear(CbhgModel& m, const float* mels, int B, int T, float* linear, float* kpart, long kpart_floats,
                 hipStream_t s);

}  // namespace tt2
