"""Shared test helpers: configs, seeded synthetic inputs, oracle hparams."""
import numpy as np  # noqa: F401

from oracle.hp import oracle_hp, wavenet_oracle_hp  # noqa: F401
from tt2.hparams import bench_wavenet_hparams, hparams
from tt2.synthetic import mol_uniforms, prenet_masks, tacotron_inputs  # noqa: F401


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


def small_wavenet_hparams(layers=6, stacks=2):
    hp = bench_wavenet_hparams()
    hp.override_from_dict(dict(layers=layers, stacks=stacks, wavenet_num_gpus=1))
    return hp


