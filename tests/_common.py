"""Shared test helpers: configs, seeded synthetic inputs, oracle hparams."""
import numpy as np

from tt2.hparams import bench_wavenet_hparams, hparams


def small_hparams():
    """Shrunken Tacotron-2 (same topology, narrow widths) so the oracle runs in seconds."""
    hp = hparams.copy()
    hp.override_from_dict(dict(
        embedding_dim=64, enc_conv_channels=64, encoder_lstm_units=32, attention_dim=32,
        attention_filters=8, prenet_layers=[32, 32], decoder_lstm_units=64, postnet_channels=64,
        style_embed_depth=64, style_att_dim=32, reference_filters=[8, 8, 16, 16, 32, 32],
        reference_depth=32, tacotron_num_gpus=1, synthesis_constraint=False))
    return hp


def full_hparams():
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    return hp


def oracle_hp(hp, synthesis_constraint=False):
    return dict(zoneout=hp.tacotron_zoneout_rate, num_mels=hp.num_mels,
                max_abs_value=hp.max_abs_value, lower_bound_decay=hp.lower_bound_decay,
                clip_outputs=hp.clip_outputs, stop_at_any=hp.stop_at_any,
                mask_encoder=hp.mask_encoder, cumulative=hp.cumulative_weights,
                synthesis_constraint=synthesis_constraint,
                synthesis_constraint_type=hp.synthesis_constraint_type,
                attention_win_size=hp.attention_win_size, num_heads=hp.num_heads)


def wavenet_oracle_hp(hp):
    return dict(layers=hp.layers, stacks=hp.stacks, residual_channels=hp.residual_channels,
                legacy=hp.legacy, residual_legacy=hp.residual_legacy,
                log_scale_min=hp.log_scale_min, upsample_scales=list(hp.upsample_scales),
                freq_axis_kernel_size=hp.freq_axis_kernel_size, max_abs_value=hp.max_abs_value,
                kernel_size=hp.kernel_size)


def small_wavenet_hparams(layers=6, stacks=2):
    hp = bench_wavenet_hparams()
    hp.override_from_dict(dict(layers=layers, stacks=stacks, wavenet_num_gpus=1))
    return hp


def tacotron_inputs(B, T, T_ref, seed=1234, ragged=True, num_mels=80):
    """ids rng(seed).integers(2,66) + EOS (id 1), pad 0; lengths; ref mels U[-4,4] (BASELINE)."""
    rng = np.random.default_rng(seed)
    ids = np.zeros((B, T), np.int32)
    if ragged:
        lengths = rng.integers(max(2, T // 2), T + 1, B).astype(np.int32)
        lengths[0] = T
    else:
        lengths = np.full(B, T, np.int32)
    for b in range(B):
        L = lengths[b]
        ids[b, :L - 1] = rng.integers(2, 66, L - 1)
        ids[b, L - 1] = 1
    ref_e = rng.uniform(-4, 4, (B, T_ref, num_mels)).astype(np.float32)
    ref_s = rng.uniform(-4, 4, (B, T_ref, num_mels)).astype(np.float32)
    return ids, lengths, ref_e, ref_s


def prenet_masks(n, B, P, seed=5339):
    return (np.random.default_rng(seed).random((n, 2, B, P)) < 0.5).astype(np.uint8)


def mol_uniforms(T, B, nr=10, seed=5339):
    rng = np.random.default_rng(seed)
    um = rng.uniform(1e-5, 1 - 1e-5, (T, B, nr)).astype(np.float32)
    ul = rng.uniform(1e-5, 1 - 1e-5, (T, B)).astype(np.float32)
    return um, ul
