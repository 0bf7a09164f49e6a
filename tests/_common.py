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




# configs[3] at the fork-default Tacotron widths: three ~135-200 character
# sentences through the text frontend, reference mels of 120 frames, the stop bias lowered so no row
# stops inside n steps (every row keeps n frames, the WaveNet leg runs over a known length)
FORK_E2E_TEXTS = [
    "The quick brown fox jumps over the lazy dog while 42 bakers on Baker St. sell $3.50 loaves of "
    "bread to every passer-by who happens to wander along the river bank at dawn.",
    "Dr. Who said that it costs 1,250 dollars to travel through time, although most of his "
    "companions insist that the true price of each journey is paid in memories and lost afternoons.",
    "Turn left at the second light, then keep going for about three miles until you see a red barn "
    "with a weathervane shaped like a rooster.",
    "It was the best of times, it was the worst of times, it was the age of wisdom, it was the age "
    "of foolishness, and it was, above all, a season of light.",
]
STOP_BIAS = ("Tacotron_model/inference/decoder/stop_token_projection/"
             "projection_stop_token_projection/bias")


def fork_e2e_case(n, B=3, seed=5339):
    """(hp, W, WW, ids, lens, ref_emt, ref_spk, prenet_masks, u_mix, u_log) of configs[3] at the
    fork widths (tt2.e2e.e2e_hparams: fork Tacotron, paper 24-layer MoL WaveNet at R=64)."""
    from tacotron.utils.text import text_to_sequence
    from tt2.e2e import e2e_hparams
    from tt2.weights import init_tacotron_weights, init_wavenet_weights
    hp = e2e_hparams(n)
    W = init_tacotron_weights(hp, seed=seed)
    W[STOP_BIAS] = np.full((1,), -6.0, np.float32)
    WW = init_wavenet_weights(hp, seed=seed)
    seqs = [text_to_sequence(t, ["english_cleaners"]) for t in FORK_E2E_TEXTS[:B]]
    T_in = max(len(s) for s in seqs)
    ids = np.zeros((B, T_in), np.int32)
    for b, s in enumerate(seqs):
        ids[b, :len(s)] = s
    lens = np.asarray([len(s) for s in seqs], np.int32)
    rng = np.random.default_rng(11)
    re = rng.uniform(-4, 4, (B, 120, 80)).astype(np.float32)
    rs = rng.uniform(-4, 4, (B, 120, 80)).astype(np.float32)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=4)
    um, ul = mol_uniforms(n * 275, B, seed=9)
    return hp, W, WW, ids, lens, re, rs, masks, um, ul
