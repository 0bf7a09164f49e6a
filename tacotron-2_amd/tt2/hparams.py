"""Hyper-parameters of the synthesis path, same names and values as the reference.

``hparams`` mirrors the fork's ``code/hparams.py:12-402`` (tf.contrib.training.HParams) and
``paper_hparams`` mirrors ``code/paper_hparams.py:5-371`` with the 17 fork-only keys the fork's
model code reads back-filled from ``hparams.py``.  Only keys that touch the
synthesis path (or the harness's I/O contract) are kept; ``parse("k=v,...")`` behaves like
``HParams.parse`` (used by ``code/train.py:35``, ``code/synthesize.py:15``).
"""
import ast
import copy

import numpy as np


class HParams(object):
    """Minimal tf.contrib.training.HParams: attribute access, values(), parse(), override."""

    def __init__(self, **kwargs):
        object.__setattr__(self, "_values", dict(kwargs))

    def __getattr__(self, name):
        try:
            return self._values[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        self._values[name] = value

    def values(self):
        return dict(self._values)

    def get(self, name, default=None):
        return self._values.get(name, default)

    def copy(self):
        return HParams(**copy.deepcopy(self._values))

    def override_from_dict(self, d):
        for k, v in d.items():
            if k not in self._values:
                raise ValueError("Unknown hyperparameter: {}".format(k))
            self._values[k] = v
        return self

    def parse(self, values):
        """Parse 'name=value,name2=[1,2],...' like HParams.parse (type follows the default)."""
        if not values:
            return self
        parts, depth, cur = [], 0, ""
        for ch in values:
            if ch in "[(":
                depth += 1
            elif ch in "])":
                depth -= 1
            if ch == "," and depth == 0:
                parts.append(cur)
                cur = ""
            else:
                cur += ch
        if cur.strip():
            parts.append(cur)
        for p in parts:
            if "=" not in p:
                raise ValueError("Could not parse hparam '{}' in {}".format(p, values))
            k, v = p.split("=", 1)
            k, v = k.strip(), v.strip()
            if k not in self._values:
                raise ValueError("Unknown hyperparameter: {}".format(k))
            old = self._values[k]
            if isinstance(old, bool):
                nv = v.lower() in ("true", "1")
            elif isinstance(old, (list, tuple)):
                nv = type(old)(ast.literal_eval(v))
            elif isinstance(old, int) and not isinstance(old, bool):
                nv = int(v)
            elif isinstance(old, float):
                nv = float(v)
            elif old is None:
                try:
                    nv = ast.literal_eval(v)
                except (ValueError, SyntaxError):
                    nv = v
            else:
                nv = v.strip("'\"")
            self._values[k] = nv
        return self


_FORK = dict(
    cleaners="english_cleaners",
    tacotron_num_gpus=4, tacotron_batch_size=96, wavenet_num_gpus=1, split_on_cpu=True,
    # audio (hparams.py:71-135)
    num_mels=80, num_freq=1025, n_fft=2048, hop_size=200, win_size=800, sample_rate=16000,
    frame_shift_ms=None, preemphasize=True, preemphasis=0.97,
    signal_normalization=True, allow_clipping_in_normalization=True, symmetric_mels=True,
    max_abs_value=4.0, normalize_for_wavenet=True, clip_for_wavenet=True, wavenet_pad_sides=1,
    min_level_db=-100, ref_level_db=20, fmin=55, fmax=7600, power=1.5, griffin_lim_iters=60,
    magnitude_power=2.0, use_lws=False,
    GL_on_GPU=True,
    # GST (hparams.py:108-115)
    use_gst=True, num_gst=10, num_heads=4, style_embed_depth=256,
    reference_filters=[32, 32, 64, 64, 128, 128], reference_depth=128,
    style_att_type="mlp_attention", style_att_dim=128,
    # Tacotron (hparams.py:140-194)
    outputs_per_step=1, stop_at_any=False, batch_norm_position="after", clip_outputs=True,
    lower_bound_decay=0.1, embedding_dim=512, enc_conv_num_layers=3, enc_conv_kernel_size=(5,),
    enc_conv_channels=512, encoder_lstm_units=256, smoothing=False, attention_dim=128,
    attention_filters=32, attention_kernel=(31,), cumulative_weights=True,
    synthesis_constraint=True, synthesis_constraint_type="window", attention_win_size=7,
    prenet_layers=[256, 256], decoder_layers=2, decoder_lstm_units=1024, max_iters=1000,
    postnet_num_layers=5, postnet_kernel_size=(5,), postnet_channels=512,
    mask_encoder=True, mask_decoder=False, predict_linear=False,
    cbhg_kernels=8, cbhg_conv_channels=128, cbhg_pool_size=2, cbhg_projection=256,
    cbhg_projection_kernel_size=3, cbhg_highwaynet_layers=4, cbhg_highway_units=128,
    cbhg_rnn_units=128,
    tacotron_zoneout_rate=0.1, tacotron_dropout_rate=0.5,
    tacotron_random_seed=5339, tacotron_data_random_state=1234,
    tacotron_synthesis_batch_size=1, tacotron_spk_emb_dim=1024, tacotron_se_concat=True,
    tacotron_use_style_emb_disc=True, tacotron_style_emb_disc_refnet=True,
    tacotron_use_orthog_loss=True,
    # Tacotron training (hparams.py:44,272-302)
    tacotron_decay_learning_rate=True, tacotron_start_decay=15000,
    tacotron_decay_steps=10000, tacotron_decay_rate=0.5, tacotron_initial_learning_rate=1e-3,
    tacotron_final_learning_rate=1e-4, tacotron_adam_beta1=0.9, tacotron_adam_beta2=0.999,
    tacotron_adam_epsilon=1e-6, tacotron_reg_weight=1e-6, tacotron_scale_regularization=False,
    tacotron_clip_gradients=True, tacotron_teacher_forcing_mode="constant",
    tacotron_teacher_forcing_ratio=1.0, cross_entropy_pos_weight=1,
    # teacher-forcing schedule (hparams.py:302-307) and natural eval (hparams.py:292)
    tacotron_teacher_forcing_init_ratio=1.0, tacotron_teacher_forcing_final_ratio=0.0,
    tacotron_teacher_forcing_start_decay=10000, tacotron_teacher_forcing_decay_steps=40000,
    tacotron_teacher_forcing_decay_alpha=None, tacotron_teacher_forcing_decay_exp_rate=0.1,
    tacotron_natural_eval=True,
    # WaveNet (hparams.py:207-253)
    input_type="raw", quantize_channels=2 ** 16, use_bias=True, legacy=True, residual_legacy=True,
    log_scale_min=float(np.log(1e-14)), log_scale_min_gauss=float(np.log(1e-7)), cdf_loss=False,
    out_channels=2, layers=20, stacks=2, residual_channels=128, gate_channels=256,
    skip_out_channels=128, kernel_size=3, cin_channels=80, upsample_type="SubPixel",
    upsample_activation="Relu", upsample_scales=[11, 25], freq_axis_kernel_size=3,
    leaky_alpha=0.4, NN_init=True, NN_scaler=0.3, gin_channels=-1, use_speaker_embedding=False,
    n_speakers=5, wavenet_random_seed=5339, wavenet_synthesis_batch_size=20, wavenet_dropout=0.05,
    wavenet_weight_normalization=False, wavenet_synth_debug=False,
    wavenet_debug_wavs=['training_data/audio/audio-LJ001-0008.npy'],
    wavenet_debug_mels=['training_data/mels/mel-LJ001-0008.npy'],
)

#: fork default hyper-parameters (code/hparams.py)
hparams = HParams(**_FORK)

_PAPER_OVERRIDES = dict(
    tacotron_num_gpus=1, hop_size=275, win_size=1100, sample_rate=22050, preemphasize=False,
    fmin=75, stop_at_any=True, synthesis_constraint=False, max_iters=10000,
    legacy=False, residual_legacy=False, log_scale_min_gauss=float(np.log(9.1188196 * 1e-4)),
    cdf_loss=True, out_channels=30, layers=24, stacks=4, residual_channels=256, gate_channels=512,
    skip_out_channels=256, upsample_type="2D", upsample_scales=[5, 5, 11], NN_scaler=0.1,
    use_speaker_embedding=True,
)

#: code/paper_hparams.py values, fork-only keys back-filled from code/hparams.py
paper_hparams = HParams(**dict(_FORK, **_PAPER_OVERRIDES))


def get_hop_size(hp):
    """datasets/audio.py get_hop_size: hop_size, or frame_shift_ms·sample_rate/1000."""
    if hp.hop_size is None:
        assert hp.frame_shift_ms is not None
        return int(hp.frame_shift_ms / 1000 * hp.sample_rate)
    return hp.hop_size


def bench_wavenet_hparams():
    """BASELINE.json config 3: paper_hparams WaveNet (24 layers / 4 stacks, 10-mix MoL, 2D
    upsampling [5,5,11], hop 275, 22.05 kHz) at residual width R=64 (G=128, S=64)."""
    return paper_hparams.copy().override_from_dict(
        dict(residual_channels=64, gate_channels=128, skip_out_channels=64))
