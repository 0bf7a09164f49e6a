/*
 * tt2.h — C ABI of libtt2.so, the MI355X (gfx950) Tacotron-2 decoder + WaveNet MoL vocoder
 * synthesis path.
 *
 * The reference (mwhitehill/Tacotron-2, TF 1.x) has no FFI: its seams are Python objects that
 * build a TF graph.  Each entry point below replaces one of those seams; the
 * Python shim in tacotron-2_amd/{tacotron,wavenet_vocoder}/ binds them with ctypes and keeps the
 * reference's class/method names.  Reference paths are relative to the reference's code/ dir.
 *
 * Conventions
 *  - Every pointer argument of a non-_dev function is HOST memory owned by the caller; the
 *    library copies in/out.  *_dev functions take DEVICE pointers and a hipStream_t (passed as
 *    void*) and enqueue asynchronously on that stream (zero-copy from torch tensors).
 *  - All arithmetic is IEEE fp32 (the reference's dtype); ids/lengths int32.
 *  - One context per device; a context is NOT thread-safe, distinct contexts are independent.
 *  - No exception crosses the ABI: every function returns a tt2_status; the message of the last
 *    failure on the calling thread is returned by tt2_last_error().
 */
#ifndef TT2_H
#define TT2_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int tt2_status;
#define TT2_OK 0
#define TT2_ERR_INVALID_ARG (-1)
#define TT2_ERR_SHAPE_MISMATCH (-2)
#define TT2_ERR_OOM (-3)
#define TT2_ERR_HIP (-4)
#define TT2_ERR_NOT_LOADED (-5)  /* a required weight was never loaded / finalize not called */
#define TT2_ERR_STATE (-6)       /* call order violated (e.g. decode before encode) */

/* Thread-local message of the last failing call on this thread ("" if none). */
const char* tt2_last_error(void);
/* Process exit guard for profiled runs (not part of any reference interface).  install = 1
 * registers an atexit handler that flushes stdio and _exit()s with the last `status` passed here
 * (1 until the caller reports success), skipping the handlers registered before it -- the HIP
 * runtime's static teardown.  Call it after the HIP runtime is loaded and before the first device
 * call, so a profiler that registers its finalisation at HSA initialisation still runs first:
 * under rocprofv3, after the tool's finalisation, the runtime's exit-time teardown of the
 * cooperative-launch queue faults inside libhsa-runtime64. */
void tt2_exit_guard(int install, int status);
/* Library / kernel build identification string (arch, version). */
const char* tt2_version(void);

/* ------------------------------------------------------------------------------------------ */
/* Tacotron-2 (replaces tacotron/models/tacotron.py Tacotron.initialize synthesis graph,       */
/* tacotron.py:31-381, and the per-step TacotronDecoderCell, Architecture_wrappers.py:197-267) */
/* ------------------------------------------------------------------------------------------ */

typedef struct tt2_config {
  /* hparams (code/hparams.py); names mirror the reference */
  int num_mels;            /* 80 */
  int n_symbols;           /* 66, tacotron/utils/symbols.py:17 */
  int embedding_dim;       /* 512 */
  int enc_conv_num_layers; /* 3 */
  int enc_conv_kernel_size;/* 5 */
  int enc_conv_channels;   /* 512 */
  int encoder_lstm_units;  /* 256 per direction */
  int attention_dim;       /* 128 */
  int attention_filters;   /* 32 */
  int attention_kernel;    /* 31 */
  int prenet_units;        /* 256 (two layers, prenet_layers=[256,256]) */
  int decoder_lstm_units;  /* 1024 (two layers) */
  int postnet_num_layers;  /* 5 */
  int postnet_kernel_size; /* 5 */
  int postnet_channels;    /* 512 */
  int use_gst;             /* 1: refnet_emt/spk + GST MultiheadAttention (tacotron.py:219-308) */
  int emt_only;            /* args.emt_only: only the emotion reference path */
  int num_gst;             /* 10 */
  int num_heads;           /* 4 */
  int style_embed_depth;   /* 256 */
  int style_att_dim;       /* 128 */
  int reference_depth;     /* 128 */
  int reference_filters[6];/* 32,32,64,64,128,128 */
  float zoneout;           /* tacotron_zoneout_rate 0.1 */
  float max_abs_value;     /* 4 */
  float lower_bound_decay; /* 0.1 */
  int symmetric_mels;      /* 1 */
  int clip_outputs;        /* 1 */
  int stop_at_any;         /* 0 (fork) / 1 (paper): identical at r = 1 -- every row's round(stop) == 1
                            * (helpers.py:40-54 reduce the batch axis of the [B, r] flags first, then
                            * any / all over the r frames); 2 = never stop before max_iters (the row
                            * chunks of a batch > 32, whose one stop step the host takes over all chunks) */
  int mask_encoder;        /* 1 */
  int cumulative_weights;  /* 1 */
  int synthesis_constraint;/* args.synth_constraint (attention.py:166, tacotron.py:315) */
  int constraint_monotonic;/* 0 = 'window', 1 = 'monotonic' */
  int attention_win_size;  /* 7 */
  /* capacity of the context (device buffers are sized once at tt2_create) */
  int max_batch;           /* <= 32 on this build */
  int max_T_in;            /* longest character sequence incl. EOS */
  int max_T_ref;           /* longest reference mel (frames) */
  int max_iters;           /* decoder step capacity (hparams.max_iters) */
  /* Tacotron_emt_attn (tacotron_emt_attn.py, chosen by args.emt_attn at synthesizer.py:24):
   * memory = encoder outputs only, no GST; the decoder attends every step over the emotion
   * reference encoder's outputs (or 24 style tokens) and feeds that context to LSTM-1
   * (Architecture_wrappers.py:203-211, 228-240).  use_gst is ignored when emt_attn != 0. */
  int emt_attn;            /* args.attn: 0 = Tacotron model, 1 'simple', 2 'multihead', 3 'style_tokens' */
  int emt_ref_gru;         /* args.emt_ref_gru: 0 'none', 1 'gru', 2 'gru_multi' (modules.py:35-55) */
  int n_emt;               /* style_tokens: one-hot emotion label width (synthesizer.py:45: 4) */
  /* style path of the Tacotron model (tacotron.py:236-308): 0 GST over style tokens (fork default),
   * 1 the 128-wide reference embeddings themselves (args.pretrained_emb_disc_all; use_gst=0 implies
   * it), 2 ReferenceEncoderAdaIn (args.adain: one shared 'refnet', both mels, D_mem = 2U + 128) */
  int style_mode;
  /* predict_linear post-processing net (CBHG, modules.py:125-184 + FrameProjection(num_freq); the
   * reference's caller is commented out at tacotron.py:466-478): weights loaded when set */
  int predict_linear;
  int num_freq;                 /* 1025 */
  int cbhg_kernels;             /* 8: conv bank kernel sizes 1..K */
  int cbhg_conv_channels;       /* 128 */
  int cbhg_pool_size;           /* 2 */
  int cbhg_projection;          /* 256 (the second projection is num_mels) */
  int cbhg_projection_kernel_size; /* 3 */
  int cbhg_highwaynet_layers;   /* 4 */
  int cbhg_highway_units;       /* 128 */
  int cbhg_rnn_units;           /* 128 per direction */
  /* hp.smoothing (attention.py:71-80,150): a = sigmoid(e) / sum_j sigmoid(e) instead of softmax
   * (Chorowski et al. 2015); masked scores (-inf / -2^32+1) get sigmoid = 0.  Launch path only: a
   * context with it set never takes the persistent decoder. */
  int smoothing;                /* 0 */
  /* hparams.outputs_per_step r (hparams.py:140; tacotron.py:322-324): each decoder step projects
   * r frames and r stop tokens, feeds the last frame back (helpers.py:57) and, with GTA targets,
   * takes every r-th target frame (helpers.py:78).  max_iters stays the decoder-STEP capacity:
   * tt2_decode's frames are [B][max_iters * r][num_mels], stop [B][max_iters * r], alignments
   * [B][T_in][max_iters] and *n_steps counts steps (n_steps * r frames are valid).  r > 1 decodes
   * on the per-step launch path; tt2_decoder_step serves r = 1 only.  1 <= r <= 8. */
  int outputs_per_step;         /* 1 */
} tt2_config;

typedef struct tt2_ctx tt2_ctx;

/* Fill *cfg with the fork defaults of code/hparams.py and the given capacities. */
void tt2_default_config(tt2_config* cfg, int max_batch, int max_T_in, int max_T_ref, int max_iters);

tt2_status tt2_create(const tt2_config* cfg, int hip_device, tt2_ctx** out);
void tt2_destroy(tt2_ctx* ctx);

/* Load one variable by its TF name (e.g. "Tacotron_model/inference/inputs_embedding"), shape as
 * in the TF graph (row-major).  Replaces tf.train.Saver.restore (tacotron/synthesizer.py:93-94). */
tt2_status tt2_load_tensor(tt2_ctx* ctx, const char* tf_name, const float* host,
                           const int64_t* shape, int ndim);
/* Check every variable is present, repack into the kernels' HBM layouts, upload. */
tt2_status tt2_finalize_weights(tt2_ctx* ctx);

/* Encoder + reference encoders + GST + attention memory/keys (tacotron.py:215-308 and TF
 * BahdanauAttention _prepare_memory).  ids [B,T_in] int32 (pad 0), lengths [B];
 * ref mels [B,T_ref,80] (pad -max_abs_value, tacotron/synthesizer.py:343-352).
 * Optional outputs: memory_out [B,T_in,D_mem] (the masked attention values), style_out
 * [B, style width]. */
tt2_status tt2_encode(tt2_ctx* ctx, const int32_t* ids, const int32_t* lengths, int B, int T_in,
                      const float* ref_emt, int T_ref_emt, const float* ref_spk, int T_ref_spk,
                      float* memory_out, float* style_out);

/* Autoregressive decoder loop: tf.contrib.seq2seq.dynamic_decode over CustomDecoder
 * (tacotron.py:349-354, custom_decoder.py:107-139) with TacoTestHelper (helpers.py:6-59), or
 * with the GTA TacoTrainingHelper (helpers.py:62-133, ratio 1) when targets != NULL.
 *   prenet_masks [max_iters,2,B,prenet_units] uint8 keep bits of the always-on prenet dropout
 *                (modules.py:355-356); NULL = counter-based device RNG keyed by seed.
 *   targets      [B,T_targets,80] teacher frames (GTA) or NULL; with r = outputs_per_step the
 *                decode runs T_targets / r steps fed by frames r-1, 2r-1, ... (helpers.py:78).
 *   frames [B,max_iters*r,80], stop [B,max_iters*r] (sigmoid probs), align [B,T_in,max_iters]
 *   (nullable) are written for steps [0, *n_steps), i.e. frames [0, *n_steps * r). */
tt2_status tt2_decode(tt2_ctx* ctx, int max_iters, const uint8_t* prenet_masks, uint64_t seed,
                      const float* targets, int T_targets, float* frames, float* stop,
                      float* align, int32_t* n_steps);

/* Read-back of the device RNG tt2_decode draws its prenet keep bits from when prenet_masks is NULL:
 * out [max_iters,2,B,prenet_units] = exactly the bits tt2_decode(..., NULL, seed, ...) uses for a
 * context of batch B (same device function).  Parity/diagnostic: re-injecting them must reproduce
 * the seeded run bit for bit. */
tt2_status tt2_prenet_keep_bits(uint64_t seed, int max_iters, int B, int prenet_units, uint8_t* out);

/* TacotronDecoderState (Architecture_wrappers.py:158-195) as caller-owned host arrays, B and T_in
 * from the last tt2_encode: cell_state = ((c1, h1), (c2, h2)) of the two ZoneoutLSTM layers (the
 * carried zoneout mix), attention = the context [B,D_mem], alignments [B,T_in] = the attention
 * state (cumulated when cumulative_weights), max_attentions [B], time.  zero_state = all zeros. */
typedef struct tt2_decoder_state {
  float* h1; float* c1;      /* [B, decoder_lstm_units] */
  float* h2; float* c2;      /* [B, decoder_lstm_units] */
  float* attention;          /* [B, D_mem] */
  float* alignments;         /* [B, T_in] */
  int32_t* max_attentions;   /* [B] */
  int32_t time;
} tt2_decoder_state;

/* One TacotronDecoderCell.__call__(inputs, state) -> ((frames, stop), next_state)
 * (Architecture_wrappers.py:197-267) on the memory of the last tt2_encode: frame_in [B,80] = the
 * cell input (GO frame = zeros, then the previous raw frame, helpers.py:57), prenet_masks [2,B,P]
 * uint8 keep bits of this step; writes state_out (arrays may alias state_in's),
 * frame_out [B,80], stop_out [B] (sigmoid), alignments_out [B,T_in] (nullable; the step's
 * alignments before accumulation).  Plain fp32 kernels: the parity / debugging seam, not the fast
 * path (tt2_decode runs the fused loop). */
tt2_status tt2_decoder_step(tt2_ctx* ctx, const float* frame_in, const uint8_t* prenet_masks,
                            const tt2_decoder_state* state_in, tt2_decoder_state* state_out,
                            float* frame_out, float* stop_out, float* alignments_out);

/* linear_outputs = clip(FrameProjection(num_freq)(CBHG(mel_outputs, None))) (tacotron.py:466-481,
 * commented out in the reference; needs predict_linear): mels [B,T,num_mels] -> linear_out
 * [B,T,num_freq] (host), or device pointers on `stream`. */
tt2_status tt2_linear_outputs(tt2_ctx* ctx, const float* mels, int B, int T, float* linear_out);
tt2_status tt2_linear_outputs_dev(tt2_ctx* ctx, const float* mels_d, int B, int T, float* linear_d, void* stream);

/* Tacotron_emt_attn: emotion labels [B] int32 of the next tt2_encode (the emt_labels placeholder,
 * synthesizer.py:35, one-hot in the style_tokens query, Architecture_wrappers.py:236; an
 * out-of-range label is a zero one-hot row like tf.one_hot).  Persist until set again. */
tt2_status tt2_set_emt_labels(tt2_ctx* ctx, const int32_t* labels, int B);
/* Tacotron_emt_attn: emotion attention weights of the last decode (tower_alignments_emt,
 * tacotron_emt_attn.py / Architecture_wrappers.py:251) as out[n_steps][B][heads][T_v]; *heads and
 * *T_v receive the shape (out may be NULL to query it after tt2_encode). */
tt2_status tt2_emt_alignments(tt2_ctx* ctx, float* out, int32_t* heads, int32_t* T_v);

/* decoder clip + Postnet + postnet_projection + final clip (tacotron.py:362-381) on the frames of
 * the last tt2_decode (frames_in == NULL: T = n_steps * outputs_per_step) or on caller frames
 * [B,T,80] (T <= max_iters * outputs_per_step).  decoder_output (nullable) and mel_out are [B,T,80]. */
tt2_status tt2_postnet(tt2_ctx* ctx, const float* frames_in, int B, int T, float* decoder_output,
                       float* mel_out);

/* encode + decode + postnet on DEVICE pointers, enqueued on `stream` (hipStream_t as void*);
 * intermediates stay in HBM.  n_steps_host receives the decoded length in steps; mel_d holds
 * [B][n_steps * r][80] (row stride n_steps * r frames), stop_d [B][max_iters * r]. */
tt2_status tt2_synthesize_dev(tt2_ctx* ctx, const int32_t* ids_d, const int32_t* lengths_d,
                              const int32_t* lengths_host, int B, int T_in,
                              const float* ref_emt_d, int T_ref_emt, const float* ref_spk_d,
                              int T_ref_spk, int max_iters, const uint8_t* prenet_masks_d,
                              uint64_t seed, float* mel_d, float* stop_d, int32_t* n_steps_host,
                              void* stream);

/* get_output_lengths (tacotron/synthesizer.py:384-387) on device: lengths_d[b] = first step
 * t < n_steps whose stop probability rounds to 1 (np.round: half-to-even), else n_steps.
 * stop_d is [B, ld] (row stride ld >= n_steps, e.g. the stop_d of tt2_synthesize_dev with
 * ld = max_iters).  Enqueued on `stream`. */
tt2_status tt2_output_lengths_dev(const float* stop_d, int B, int n_steps, int ld,
                                  int32_t* lengths_d, void* stream);

/* Measurement hooks (not part of the reference surface; used by bench.py for the roofline).
 * tt2_last_timings: HIP-event times (ms) of the last tt2_synthesize_dev phases
 *   [encode, decode loop, postnet].
 * tt2_profile_decoder_kernels: after a decode, re-launch each per-step decoder kernel `iters`
 *   times back-to-back on the context stream between one HIP event pair; avg_us[10] = time per
 *   launch of [prenet, lstm(layer1/layer2 alternating), query, energy(+side job), softmax+context
 *   (+side job), frame/stop projection, lstm layer 2 only, side job alone, energy alone,
 *   softmax+context alone].  Leaves the decoder state undefined. */
tt2_status tt2_last_timings(tt2_ctx* ctx, float* ms3);
tt2_status tt2_profile_decoder_kernels(tt2_ctx* ctx, int iters, float* avg_us10);
/* s_memtime phase stamps (block 0) recorded during the last tt2_profile_decoder_kernels call:
 * [0..5] prenet, [8..12] energy, [16..19] lstm; or, after a persistent decode run with env
 * TT2_STAMP_STEP=k, s_memrealtime (100 MHz) stamps [0..15] of work-group 0's stages at step k.
 * Diagnostic only. */
tt2_status tt2_debug_stamps(tt2_ctx* ctx, long long* out64);
/* Which decoder implementation the context uses for its current shapes: *persistent = 1 for the
 * single-launch persistent kernel (k_decode_persist: fork-default widths, B <= 32, T_in <= 256,
 * a device with >= 256 CUs; env TT2_DECODER=launch forces 0), 0 for the per-step launch path;
 * *kernel_ms = HIP-event duration of the last persistent decode launch (0 otherwise). */
tt2_status tt2_decoder_path(tt2_ctx* ctx, int* persistent, float* kernel_ms);
/* Persistent decode run with env TT2_STAMP_STEP=k: s_memrealtime (100 MHz) stamps [256 work-groups]
 * [32 stage points] of step k (k_decode_persist PD_STAMP sites).  Diagnostic only. */
tt2_status tt2_debug_pd_stamps(tt2_ctx* ctx, long long* out8192);
/* Measured HBM bandwidth of this device (the spec peak confirmed on the box): a
 * STREAM-like copy between two `bytes`-sized device buffers (choose >> the 256 MB MALL), 16-byte
 * loads/stores; *gbps = (read + write bytes) / the best of `iters` timed copies, in GB/s.  No
 * reference counterpart (measurement only). */
tt2_status tt2_hbm_copy_gbps(int hip_device, long long bytes, int iters, double* gbps);

/* ------------------------------------------------------------------------------------------ */
/* WaveNet MoL vocoder (replaces wavenet_vocoder/models/wavenet.py WaveNet.initialize synthesis */
/* branch :408-465 and WaveNet.incremental :724-911)                                           */
/* ------------------------------------------------------------------------------------------ */

typedef struct tt2_wn_config {
  int layers;              /* 24 */
  int stacks;              /* 4 */
  int residual_channels;   /* R */
  int gate_channels;       /* G = 2R */
  int skip_out_channels;   /* S */
  int kernel_size;         /* 3 */
  int cin_channels;        /* 80 */
  int out_channels;        /* 30 = 3 * nr_mix (MoL head) or 2 (Gaussian head, gaussian.py:39-52) */
  int legacy;              /* skip-sum sqrt(1/2) scaling (wavenet.py:833-836) */
  int residual_legacy;     /* residual sqrt(1/2) scaling (modules.py:517-520) */
  float log_scale_min;     /* log(1e-14) */
  int n_upsample;          /* number of ConvTranspose2D layers */
  int upsample_scales[8];  /* [5,5,11] */
  int freq_axis_kernel_size; /* 3 */
  int max_batch;
  int64_t max_samples;     /* capacity in audio samples per utterance */
  int upsample_type;       /* 0 '2D' (paper), 1 '1D', 2 'Resize', 3 'SubPixel' (fork default),
                              4 'NearestNeighbor' (wavenet.py:163-203) */
  int upsample_activation; /* 0 None, 1 'Relu', 2 'LeakyRelu' (wavenet.py:195-201) */
  float leaky_alpha;       /* 0.4 */
  int NN_init;             /* SubPixel: 0 = every output channel uses channel 0's kernel
                              (SubPixelConvolution.build, modules.py:585-593) */
  float log_scale_min_gauss; /* Gaussian head (out_channels == 2): log(1e-7) fork / paper value */
  int gin_channels;        /* global conditioning width (<= 0: off, the fork default -1;
                              wavenet.py:152-158, modules.py:427-433, 505-509) */
  int n_speakers;          /* > 0: use_speaker_embedding, the gc_embedding table [n_speakers, gin] */
  int input_type;          /* 0 'raw', 1 'mulaw' (scalar input), 2 'mulaw-quantize': one-hot input of
                              quantize_channels classes and the softmax head sampled by tf.multinomial
                              (wavenet.py:433-452, 861-867); out_channels must equal quantize_channels */
  int quantize_channels;   /* 256 */
} tt2_wn_config;

typedef struct tt2_wn_ctx tt2_wn_ctx;

void tt2_wn_default_config(tt2_wn_config* cfg, int max_batch, int64_t max_samples);
tt2_status tt2_wn_create(const tt2_wn_config* cfg, int hip_device, tt2_wn_ctx** out);
void tt2_wn_destroy(tt2_wn_ctx* ctx);
tt2_status tt2_wn_load_tensor(tt2_wn_ctx* ctx, const char* tf_name, const float* host,
                              const int64_t* shape, int ndim);
tt2_status tt2_wn_finalize(tt2_wn_ctx* ctx);
/* Global condition of the next generate calls (cfg.gin_channels > 0), replacing g in
 * WaveNet.incremental (wavenet.py:770-775) and the per-layer conv1x1g term added to both gate
 * halves (ResidualConv1DGLU.step, modules.py:505-509): speaker_ids [B] (int32, rows of the
 * gc_embedding table; cfg.n_speakers > 0) or features [B, gin_channels] (the g tensor itself).
 * g is constant over time, so every layer's term g·W_g + b_g is folded once into the conditioning
 * of each row.  Both NULL: clear (the row-b term then comes from no global condition, an error
 * when gin_channels > 0). */
tt2_status tt2_wn_set_global_condition(tt2_wn_ctx* ctx, const int32_t* speaker_ids,
                                       const float* features, int B);

/* Fast-WaveNet incremental synthesis of T = T_f * prod(upsample_scales) samples per row.
 *   cond     [B,T_f,cin] conditioning ALREADY clipped + _interp'd to [0,1]
 *            (wavenet_vocoder/synthesizer.py:63-70 is host-side, done by the shim).
 *   u_mix    [T,B,nr_mix], u_log [T,B]: injected uniforms of the MoL sampler (mixture.py:91,104)
 *            in [1e-5, 1-1e-5); NULL = counter-based device RNG keyed by seed.  Gaussian head:
 *            u_mix unused, u_log [T,B] = the N(0,1) draws of Normal.sample (gaussian.py:50).
 *   teacher  [B,T] or NULL: test_inputs override of the next input (wavenet.py:876-878).
 *   wav_out  [B,T]; mix_idx_out [B,T] (nullable); logits_out [B,T,out_channels] (nullable);
 *   upsampled_out [B,cin,T] (nullable, = tower_synth_upsampled_local_features). */
tt2_status tt2_wn_generate(tt2_wn_ctx* ctx, const float* cond, int B, int T_f,
                           const float* u_mix, const float* u_log, uint64_t seed,
                           const float* teacher, float* wav_out, int32_t* mix_idx_out,
                           float* logits_out, float* upsampled_out);
/* input_type 2 ('mulaw-quantize') through tt2_wn_generate / tt2_wn_generate_unconditional:
 * u_log [T,B] carries the uniforms of tf.multinomial (u_mix unused), teacher [B,T] holds class
 * indices (the one-hot test_inputs, wavenet.py:752-759), mix_idx_out the drawn classes, wav_out
 * inv_mulaw_quantize of them, logits_out [B,T,quantize_channels]. */

/* Unconditional synthesis (cin_channels <= 0, no local condition: wavenet.py:410-411 with
 * synthesis_length T): T samples per row, the same sampler / teacher / output contract as
 * tt2_wn_generate (the global condition still applies when gin_channels > 0). */
tt2_status tt2_wn_generate_unconditional(tt2_wn_ctx* ctx, int B, int64_t T, const float* u_mix,
                                         const float* u_log, uint64_t seed, const float* teacher,
                                         float* wav_out, int32_t* mix_idx_out, float* logits_out);

/* Same on DEVICE pointers, enqueued on `stream` (hipStream_t as void*).  cond_d is
 * CHANNELS-FIRST [B, cin, T_f] (the layout tt2_wn_cond_from_mels_dev writes; the reference
 * transposes to it before upsampling, wavenet.py:427). */
tt2_status tt2_wn_generate_dev(tt2_wn_ctx* ctx, const float* cond_d, int B, int T_f,
                               const float* u_mix_d, const float* u_log_d, uint64_t seed,
                               const float* teacher_d, float* wav_d, int32_t* mix_idx_d,
                               float* logits_d, void* stream);

/* WaveNet conditioning from Tacotron mels, the device half of wavenet_vocoder/synthesizer.py:56-70
 * (+ feeder.py _interp :426-428): row b of mels_d [B, ld_t, num_mels] keeps its first
 * lengths_d[b] frames, clipped to [lo, hi] if clip (clip_for_wavenet), padded with lo to T_f
 * frames (_pad_inputs with T2_output_range[0]), rescaled (x-lo)/(hi-lo) if normalize
 * (normalize_for_wavenet), written channels-first to cond_d [B, num_mels, T_f]. */
tt2_status tt2_wn_cond_from_mels_dev(const float* mels_d, int ld_t, const int32_t* lengths_d,
                                     int B, int T_f, int num_mels, float lo, float hi, int clip,
                                     int normalize, float* cond_d, void* stream);

/* HIP-event times (ms) of the last generate call: [upsample, conditioning GEMM, generation]. */
tt2_status tt2_wn_last_timings(tt2_wn_ctx* ctx, float* ms3);

/* Diagnostic: s_memrealtime (100 MHz, device-wide) stamps of utterance 0 at sample T/2 of the last
 * generate call, out512[stage*8 + k]: k=0 input received, 1..3 after each layer, 4 head done
 * (last stage), 5 sample handed to stage 0 (last stage). */
tt2_status tt2_wn_debug_stamps(tt2_wn_ctx* ctx, long long* out512);

/* Read-back of the device RNG tt2_wn_generate draws from when u_mix/u_log are NULL (same device
 * functions): u_mix [T,B,nr_mix] and u_log [T,B] of a generate call of batch B; gaussian != 0:
 * u_log = the N(0,1) draws of the Gaussian head, u_mix untouched (may be NULL). */
tt2_status tt2_wn_noise(uint64_t seed, int T, int B, int nr_mix, int gaussian, float* u_mix,
                        float* u_log);

/* Standalone sample_from_discretized_mix_logistic (mixture.py:76-107) on the current HIP device:
 * logits [n, 3*nr_mix], u_mix [n, nr_mix], u_log [n] (host) -> x [n], k [n] (host). */
tt2_status tt2_mol_sample(const float* logits, const float* u_mix, const float* u_log, int n,
                          int nr_mix, float log_scale_min, float* x, int32_t* k);

/* ------------------------------------------------------------------------------------------ */
/* Griffin-Lim vocoder, TF GPU variant (GL_on_GPU = True, hparams.py:135): replaces             */
/* datasets/audio.py inv_mel_spectrogram_tensorflow / inv_linear_spectrogram_tensorflow         */
/* (:131-143) + _griffin_lim_tensorflow (:163-176), called by tacotron/synthesizer.py:152-160    */
/* ------------------------------------------------------------------------------------------ */

typedef struct tt2_gl_config {
  int n_fft;               /* 2048 (fft_length; power of two <= 4096) */
  int hop_size;            /* 275 paper / 200 fork (frame_step) */
  int win_size;            /* 1100 paper / 800 fork (frame_length, periodic Hann window) */
  int num_mels;            /* 80 */
  float magnitude_power;   /* 2 */
  float power;             /* 1.5 (S^power before G&L) */
  float ref_level_db;      /* 20 */
  float min_level_db;      /* -100 */
  float max_abs_value;     /* 4 */
  int symmetric_mels;      /* 1 */
  int allow_clipping_in_normalization; /* 1 */
  int griffin_lim_iters;   /* 60 */
} tt2_gl_config;

typedef struct tt2_gl_ctx tt2_gl_ctx;

void tt2_gl_default_config(tt2_gl_config* cfg);
tt2_status tt2_gl_create(const tt2_gl_config* cfg, int hip_device, tt2_gl_ctx** out);
void tt2_gl_destroy(tt2_gl_ctx* ctx);
/* pinv(mel_basis) [n_fft/2+1, num_mels] row-major (_mel_to_linear_tensorflow, audio.py:237-241;
 * the mel basis is librosa.filters.mel(sr, n_fft, num_mels, fmin, fmax), audio.py:243-246). */
tt2_status tt2_gl_set_inv_mel_basis(tt2_gl_ctx* ctx, const float* inv_basis);
/* spec [T, num_mels] (is_mel = 1, normalised mel as the Tacotron emits it) or [T, n_fft/2+1]
 * (is_mel = 0, normalised linear spectrogram) -> wav_out [(T-1)*hop + win] (no inverse
 * pre-emphasis: the reference applies it on the host afterwards, synthesizer.py:153-154).
 * iters < 0 = cfg.griffin_lim_iters. */
tt2_status tt2_gl_synthesize(tt2_gl_ctx* ctx, const float* spec, int T, int is_mel, int iters,
                             float* wav_out);
/* Same on DEVICE pointers, enqueued on `stream` (hipStream_t as void*). */
tt2_status tt2_gl_synthesize_dev(tt2_gl_ctx* ctx, const float* spec_d, int T, int is_mel,
                                 int iters, float* wav_d, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Teacher-forced decoder training step (BASELINE configs[4]): replaces    */
/* Tacotron.initialize(is_training=True) + add_loss() + add_optimizer() (tacotron.py:31-35,      */
/* 683-986, 1002-1251) for the decoder slice: TacoTrainingHelper dynamic_decode (helpers.py:      */
/* 62-133) -> before-MSE + stop CE + L2 (tacotron.py:774,778-779,865-867) -> BPTT gradients ->   */
/* clip_by_global_norm(1.0) + AdamOptimizer (tacotron.py:1029,1219-1221).                        */
/* Trainable variables are the decoder's TF names (memory_layer, query_layer, location conv /    */
/* layer, v_a, b_a, prenet, both LSTM cells, frame and stop projections).                        */
/* ------------------------------------------------------------------------------------------ */

typedef struct tt2_train_config {
  int batch;               /* rows per step on this device (configs[4]: 64) */
  int max_T_in;            /* <= 320 (attention-kernel LDS budget) */
  int max_T_out;           /* frames (decoder steps · outputs_per_step) */
  int memory_dim;          /* D_mem (1024 fork default) */
  int num_mels;            /* 80 */
  int prenet_units;        /* 256 (both prenet layers) */
  int decoder_lstm_units;  /* 1024 */
  int attention_dim;       /* 128 (must divide 256) */
  int attention_filters;   /* 32 (<= 32) */
  int attention_kernel;    /* 31 */
  float zoneout;           /* 0.1: used only when no zoneout masks are passed (inference mix) */
  float reg_weight;        /* tacotron_reg_weight 1e-6 */
  float adam_beta1, adam_beta2, adam_epsilon;  /* 0.9, 0.999, 1e-6 */
  float clip_norm;         /* 1.0 (tacotron_clip_gradients); <= 0 disables */
  int precision;           /* 0 = fp32 GEMMs (parity); 1 = bf16 GEMM operands, fp32 accumulation,
                              fp32 master weights / cell state / optimizer (configs[4]) */
  int clip_outputs;        /* 1: decoder_output = clip(frames, clip_lo, clip_hi) before the loss */
  float clip_lo, clip_hi;  /* -max_abs_value - lower_bound_decay, max_abs_value (-4.1, 4) */
  int postnet;             /* 1: also the Postnet (training-mode BN + dropout) and the after loss */
  int postnet_layers, postnet_channels, postnet_kernel;  /* 5, 512, 5 */
  float bn_momentum, bn_eps;                               /* 0.99, 1e-3 (tf.layers defaults) */
  /* front end (frontend = 1): the step starts from character ids + reference mels
   * (tt2_train_forward_backward_text_dev) and also trains the encoder (embedding, 3x conv + BN +
   * ReLU + dropout, bidirectional Zoneout-LSTM), both reference encoders (6x conv2d + BN + ReLU,
   * GRU, dense tanh) and both GST attentions (tacotron.py:215-308, modules.py:9-64,251-323,
   * multihead_attention.py:35-132); memory_dim = 2*encoder_lstm_units + (emt_only ? 1 : 2) *
   * style_embed_depth */
  int frontend;
  int n_symbols, embedding_dim, enc_conv_layers, enc_conv_kernel, enc_conv_channels, encoder_lstm_units;
  int emt_only, num_gst, num_heads, style_embed_depth, style_att_dim, reference_depth;
  int reference_filters[6];
  int max_T_ref;                                           /* reference mel frames (capacity) */
  /* loss options (tacotron.py:758-767, modules.py:532-575; hparams.py:192-193): mask_decoder = 1
   * masks the before / after MSE and the stop cross entropy past each row's target length
   * (tt2_train_set_target_lengths), the stop loss then being TF's weighted cross entropy with
   * pos_weight (the unmasked stop loss ignores pos_weight, as the reference's does) */
  int mask_decoder;
  float pos_weight;
  /* style-embedding losses of the default GST training graph (frontend = 1; tacotron.py:486-495,
   * 812-820, 840-846; hparams tacotron_use_style_emb_disc / tacotron_use_orthog_loss):
   * n_emt > 0 adds Style_Emb_Disc 'style_disc_emt' (dense 128 -> n_emt) on refnet_emt's output
   * with softmax cross entropy against the emotion labels (tt2_train_set_style_labels), n_spk > 0
   * the same for refnet_spk and the speaker labels (not emt_only); orthog_weight > 0 adds
   * orthog_weight * ||refnet_emt · refnet_spkᵀ||_F (0.02 in the reference; not emt_only).  0 = off. */
  int n_emt, n_spk;
  float orthog_weight;
  /* hp.use_gst (tacotron.py:269-291): 1 = each reference embedding passes through its GST
   * multi-head attention (style_embed_depth wide); 0 = the 128-wide reference embeddings themselves
   * are the style embeddings (no style tokens / attention variables; memory_dim = 2*U + (emt_only ?
   * 1 : 2) * 128) */
  int use_gst;
  /* args.adain (tacotron.py:236-242, 266-268; modules.py:66-107): ReferenceEncoderAdaIn 'refnet' in
   * training mode -- the speaker and emotion mels through two conv2d + ReLU stacks without batch
   * norm (strides (2,2),(2,2),(1,1)x4; variables refnet/conv2d_i/conv2d/{kernel,bias} speaker, conv2d_1/{kernel,bias}
   * emotion), the speaker map restyled by the emotion map's per-channel moments, one GRU + dense
   * tanh; its 128-wide output is the style embedding (memory_dim = 2*encoder_lstm_units + 128).
   * Needs both references, no style classifiers / orthogonality loss (the reference builds none). */
  int adain;
  /* hp.smoothing (attention.py:71-91,150): the attention's probability_fn is the smoothing
   * normalisation a_j = sigmoid(e_j) / sum_k sigmoid(e_k) over the unmasked positions instead of the
   * softmax; the backward multiplies the softmax form by (1 - sigmoid(e_j)).  Runs the per-step
   * attention launches (the persistent forward keeps the softmax). */
  int smoothing;
  /* hparams.outputs_per_step r (hparams.py:140; tacotron.py:322-324; helpers.py:78,129): each decoder
   * step projects r frames (frame projection num_mels*r wide, stop projection r wide) and is fed the
   * last of the r target frames of the previous step (targets[:, r-1::r]).  T_out (the frame count of
   * targets / stop targets / postnet masks) must be a multiple of r; prenet and zoneout masks and the
   * teacher-forcing draw are per decoder step (T_out / r); alignments are [B][T_in][T_out / r]. */
  int outputs_per_step;
} tt2_train_config;

typedef struct tt2_train_ctx tt2_train_ctx;

void tt2_train_default_config(tt2_train_config* cfg, int batch, int max_T_in, int max_T_out);
tt2_status tt2_train_create(const tt2_train_config* cfg, int hip_device, tt2_train_ctx** out);
void tt2_train_destroy(tt2_train_ctx* ctx);
/* Same names/shapes as tt2_load_tensor; names outside the decoder slice are ignored. */
tt2_status tt2_train_load_tensor(tt2_train_ctx* ctx, const char* tf_name, const float* host,
                                 const int64_t* shape, int ndim);
/* All slice variables loaded -> zero the Adam moments. */
tt2_status tt2_train_finalize(tt2_train_ctx* ctx);
/* Use a caller-owned device buffer (e.g. a torch tensor RCCL all-reduces) as the flat gradient
 * buffer; NULL restores the internal one.  *n_out = its length in floats: every variable's gradient
 * followed by ONE status word that each forward_backward writes (0 = ok, 1 = the persistent forward
 * timed out in a hand-off or stopped early).  The word travels in the tower mean with the gradients,
 * and tt2_train_apply_dev skips the Adam and BN moving-average updates while it is nonzero, so a
 * failed forward on any rank leaves every rank's weights unchanged; tt2_train_losses reports it. */
tt2_status tt2_train_bind_grads_dev(tt2_train_ctx* ctx, float* grads_d, int64_t* n_out);
/* Every batch-norm moving_mean / moving_variance (Postnet, encoder convs, reference-encoder
 * convs) packed in variable order into a caller-owned device buffer (unpack = 0) or written back
 * from it (unpack = 1), enqueued on `stream`; buf_d NULL only sets *n_out = the float count.
 * Data-parallel ranks update these from their own shard's batch statistics; the host averages the
 * packed buffer over ranks after apply, where the reference's towers all update ONE shared set of
 * UPDATE_OPS variables (tacotron.py:1088-1090, tower loop 1194-1208). */
tt2_status tt2_train_moving_stats_dev(tt2_train_ctx* ctx, float* buf_d, int64_t* n_out, int unpack,
                                      void* stream);
/* Forward + losses + backward on DEVICE inputs: memory [B,T_in,D] (encoder outputs ⊕ style),
 * lengths int32 [B], mel targets [B,T_out,80], stop targets [B,T_out] (T_out frames, a multiple of
 * cfg.outputs_per_step r), prenet keep bits u8 [T_out/r,2,B,P] and zoneout keep bits u8
 * [T_out/r,4,B,H] (c1,h1,c2,h2; one set per decoder step) or NULL (inference mix),
 * Postnet dropout keep bits u8 [layers,B,T_out,channels] or NULL (no dropout; cfg.postnet only).
 * Gradients (incl. L2) land in the flat gradient buffer; enqueued on `stream`. */
tt2_status tt2_train_forward_backward_dev(tt2_train_ctx* ctx, const float* memory_d,
                                          const int32_t* lengths_d, const float* targets_d,
                                          const float* stop_targets_d,
                                          const uint8_t* prenet_masks_d,
                                          const uint8_t* zoneout_masks_d,
                                          const uint8_t* postnet_masks_d, int T_in, int T_out,
                                          void* stream);
/* The whole configs[4] step on a frontend context: ids [B,T_in] int32 (pad 0) and lengths [B],
 * reference mels ref_emt / ref_spk [B,T_ref,80] (ref_spk NULL when emt_only) -> front end in
 * training mode -> memory -> the decoder + Postnet step above -> backward through everything.
 * enc_conv_masks [enc_conv_layers,B,T_in,enc_conv_channels] u8 dropout keep bits (rate 0.5) or NULL
 * (no dropout); enc_zoneout_masks [T_in,2 (fw,bw),2 (c,h),B,encoder_lstm_units] u8 zoneout keep bits
 * by recurrence step or NULL (inference mix).  Replaces Tacotron.initialize(is_training=True) +
 * add_loss + the gradient half of add_optimizer (tacotron.py:31-35, 683-1109). */
tt2_status tt2_train_forward_backward_text_dev(tt2_train_ctx* ctx, const int32_t* ids_d,
                                               const int32_t* lengths_d, const float* ref_emt_d,
                                               const float* ref_spk_d, int T_ref,
                                               const float* targets_d, const float* stop_targets_d,
                                               const uint8_t* prenet_masks_d,
                                               const uint8_t* zoneout_masks_d,
                                               const uint8_t* postnet_masks_d,
                                               const uint8_t* enc_conv_masks_d,
                                               const uint8_t* enc_zoneout_masks_d, int T_in, int T_out,
                                               void* stream);
/* Target lengths [B] (host int32, copied) for cfg.mask_decoder: the next forward_backward calls
 * mask every loss past t >= lengths[b] (TacoTrainingHelper + MaskedMSE / MaskedSigmoidCrossEntropy,
 * tacotron.py:56,758-767).  NULL clears them; a masked context without them fails the step like
 * the reference's RuntimeError (tacotron.py:56-57). */
tt2_status tt2_train_set_target_lengths(tt2_train_ctx* ctx, const int32_t* lengths);
/* Teacher-forcing draw of the next forward_backward calls (TacoTrainingHelper.next_inputs,
 * helpers.py:122-133): feed_target[t] (host u8, one per decoder step [T_out/r], copied) = 1 feeds
 * the target frame t·r-1 to step t, 0 feeds the last of the decoder's own (unclipped) r frames of
 * step t-1, whose gradient then flows back through the prenet into that frame; feed_target[0] is
 * ignored (go frame).  It is the outcome of the
 * reference's per-step draw u < ratio (ratio: constant or _teacher_forcing_ratio_decay,
 * helpers.py:140-180), injected like the dropout keep bits.  NULL = every step teacher-forced. */
tt2_status tt2_train_set_teacher_forcing(tt2_train_ctx* ctx, const uint8_t* feed_target, int T_out);
/* Per-step emotion / speaker labels [B] of the style-embedding classifiers (feeder.emt_labels /
 * spk_labels, tacotron/train.py:127-130); both NULL clears them.  Required before a step when
 * n_emt / n_spk > 0.  An out-of-range label is tf.one_hot's zero row (loss 0). */
tt2_status tt2_train_set_style_labels(tt2_train_ctx* ctx, const int32_t* emt_labels, const int32_t* spk_labels);
/* Synchronise; out3 = {style_emb_loss_emt, style_emb_loss_spk, style_emb_orthog_loss} of the last
 * text step (zeros when off); they are part of the step's loss and gradients. */
tt2_status tt2_train_style_losses(tt2_train_ctx* ctx, float* out3);
/* clip_by_global_norm + Adam with learning rate lr at update count global_step (>= 1). */
tt2_status tt2_train_apply_dev(tt2_train_ctx* ctx, float lr, int global_step, void* stream);
/* Synchronise; out5 = {before_loss, stop_loss, reg_loss, grad_global_norm (after apply),
 * after_loss (0 without the Postnet)}; fb_ms (nullable) = device time of the last
 * forward_backward.  apply also runs the Postnet BN moving-average updates. */
tt2_status tt2_train_losses(tt2_train_ctx* ctx, float* out5, float* fb_ms);
/* which: 0 = parameter, 1 = gradient, 2 = Adam m, 3 = Adam v; name "memory" (which ignored) =
 * d loss / d memory [B,T_in,D] of the last forward_backward; on a frontend context also
 * "frontend:memory" = the memory the front end produced [B,T_in,D] and "frontend:refnet_emt" /
 * "frontend:refnet_spk" = the reference embeddings [B,128] (diagnostic read-backs); with the Postnet
 * "postnet:projection" = the Postnet projection [B,T,80] of the last forward (mel_outputs =
 * clip(decoder_output + it), tacotron.py:375-378); "diag:blas_calls"
 * = one float, the number of products routed to rocBLAS since create (bf16 mode). */
tt2_status tt2_train_get_tensor(tt2_train_ctx* ctx, const char* tf_name, int which, float* host);
/* Last forward's decoder frames [B,T,80], stop logits [B,T], alignments [B,T_in,T] (nullable). */
tt2_status tt2_train_outputs(tt2_train_ctx* ctx, float* frames, float* stop_logits,
                             float* alignments);

#ifdef __cplusplus
}
#endif
#endif /* TT2_H */
