// Tacotron_emt_attn (tacotron_emt_attn.py; chosen by synthesizer.py:24 / train.py:106 when
// args.emt_attn): the decoder attends, every step, over the emotion reference encoder's outputs
// (or over 24 learned style tokens) with its LSTM output as the query; the resulting emotion
// context joins the next step's LSTM-1 input (Architecture_wrappers.py:203-211, 228-240).
// The text encoder, location-sensitive attention, projections and Postnet are the Tacotron ones
// (tacotron.hip); this file holds only what the variant adds.
#pragma once
#include "common.h"

namespace tt2 {

enum EmtAttn { EMT_OFF = 0, EMT_SIMPLE = 1, EMT_MULTIHEAD = 2, EMT_STYLE_TOKENS = 3 };  // args.attn
enum EmtRefGru { EMT_GRU_NONE = 0, EMT_GRU_BI = 1, EMT_GRU_MULTI = 2 };                 // args.emt_ref_gru
constexpr int EMT_NTOK = 24, EMT_TOKD = 16;  // style_tokens [24, 16] (tacotron_emt_attn.py:212-214)
constexpr int EMT_NMULTI = 8;                // 'gru_multi': 8 GRU + dense(128, tanh) heads (modules.py:46)
constexpr int EMT_OUT = 128;                 // dense widths fixed by the reference (modules.py:49, Architecture_wrappers.py:234)

struct EmtModel {
  int attn = EMT_OFF, ref_gru = EMT_GRU_NONE, spk = 0, n_emt = 0;
  int H = 0;       // decoder_lstm_units (query width)
  int Aq = 0;      // attention units: attention_dim ('simple') / style_att_dim (multi-head)
  int heads = 1, dh = 0;
  int Dv = 0;      // width of one attended value row
  int XW = 0;      // LSTM-1 input columns this variant adds after [prenet | context]
  int D = 0, gin = 0, NG = 0;  // reference GRU depth, CNN output width, GRUs in refnet_emt
  int max_batch = 0, max_Tv = 0, max_iters = 0;
  int B = 0, Tv = 0;           // of the last emt_encode
  // weights (TF variables, see emt_load)
  DevBuf wq, qb, qlab, wk, bk, vv, ab, wd, bd, tokens;
  DevBuf gwx, gbx, gwhg, gwhc, gkd, gbd;
  // activations
  DevBuf xg, val, ke, qrow, labels, hist;
  bool on() const { return attn != EMT_OFF; }
  long val_bstride() const { return attn == EMT_STYLE_TOKENS ? 0 : (long)Tv * Dv; }
  long ke_bstride() const { return attn == EMT_STYLE_TOKENS ? 0 : (long)Tv * Aq; }
};

// Shapes from the config; throws on combinations the reference graph cannot build (e.g. 'simple'
// with a value width != attention_dim: its zero attention state and the later ones would differ).
void emt_configure(EmtModel& m, int attn, int ref_gru, int emt_only, int n_emt, int H, int attention_dim,
                   int style_att_dim, int num_heads, int ref_depth, int num_mels, const int filters[6],
                   int max_batch, int max_T_ref, int max_iters);
void emt_load(EmtModel& m, const WeightMap& wm, const std::string& prefix);
// Per utterance: refnet_emt's CNN output x [B][T2][gin] (null for style tokens) -> attended values,
// their keys, the per-row query bias (style tokens: + the one-hot emotion label row).
void emt_encode(EmtModel& m, const float* x, int B, int T2, hipStream_t s);
// Decode start (zero_state, Architecture_wrappers.py:182): the emotion context is zero; the
// speaker embedding part of the block is constant.  X1a / X1b: the AF LSTM-1 input buffers.
void emt_init_launch(const EmtModel& m, const float* spk, float* X1a, float* X1b, int col0, hipStream_t s);
// One step: h2 = Xp[:, 0:H] (AF) -> emotion context -> X1 columns [col0, col0 + XW) of the next
// step; alignments of step t into hist when t < max_iters.  Skipped once *done.
void emt_step_launch(const EmtModel& m, const int* done, const float* Xp, float* X1, int col0, const float* spk, int t,
                     hipStream_t s);

// TF1 GRUCell over every frame of B rows by NG independent GRUs (k_emt_gru), xg [B][T][NG][3D] the
// x products + biases: mode 0 all outputs with GRU 1 walking backwards (a full-length BiGRU,
// out [B][T][NG·D]); mode 1 last output -> dense(128, tanh) (out [B][NG][128]).  Also the CBHG's
// bidirectional GRU (cbhg.hip).
void gru_sequence(const float* xg, int B, int T, int D, int NG, const float* whg, const float* whc, int mode,
                  const float* kd, const float* bd, float* out, hipStream_t s);

}  // namespace tt2
