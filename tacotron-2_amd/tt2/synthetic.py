"""Seeded synthetic inputs of the BASELINE.json configs (no datasets are available offline)."""
import numpy as np


def tacotron_inputs(B, T, T_ref, seed=1234, ragged=True, num_mels=80):
    """Character ids rng(seed).integers(2,66) followed by EOS (id 1, tacotron/utils/text.py:40-41),
    pad id 0; lengths (ragged: U[T/2, T], row 0 full); reference mels U[-4, 4] [B, T_ref, 80]."""
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
    """Keep bits of the always-on prenet dropout (rate 0.5), [n, 2, B, P] uint8."""
    return (np.random.default_rng(seed).random((n, 2, B, P)) < 0.5).astype(np.uint8)


def mol_uniforms(T, B, nr=10, seed=5339):
    """U[1e-5, 1-1e-5) uniforms of the MoL sampler (mixture.py:91,104): u_mix [T,B,nr], u_log [T,B]."""
    rng = np.random.default_rng(seed)
    um = rng.uniform(1e-5, 1 - 1e-5, (T, B, nr)).astype(np.float32)
    ul = rng.uniform(1e-5, 1 - 1e-5, (T, B)).astype(np.float32)
    return um, ul


def train_batch(B, T_in, T_out, D, num_mels=80, seed=1234, ragged=True):
    """configs[4]-shaped synthetic teacher-forced batch: decoder memory N(0, 0.5) [B,T_in,D],
    input lengths (ragged U[T_in/2, T_in], row 0 full), mel targets U[-4, 4] [B,T_out,80] and
    stop-token targets (0 before each row's target length, 1 from it on; tacotron/feeder.py pads
    with 1), target lengths U[T_out/2, T_out] (row 0 full)."""
    rng = np.random.default_rng(seed)
    memory = (rng.standard_normal((B, T_in, D)) * 0.5).astype(np.float32)
    lengths = np.full(B, T_in, np.int32)
    tlen = np.full(B, T_out, np.int32)
    if ragged and B > 1:
        lengths[1:] = rng.integers(max(1, T_in // 2), T_in + 1, B - 1)
        tlen[1:] = rng.integers(max(1, T_out // 2), T_out + 1, B - 1)
    targets = rng.uniform(-4, 4, (B, T_out, num_mels)).astype(np.float32)
    stop = (np.arange(T_out)[None, :] >= tlen[:, None] - 1).astype(np.float32)
    return memory, lengths, targets, stop


def zoneout_masks(n, B, H, rate=0.1, seed=5339):
    """Training-mode zoneout keep bits (modules.py:236-240: dropout(new - prev, 1 - rate)) of the
    two decoder LSTMs: [n, 4, B, H] uint8 (c1, h1, c2, h2)."""
    return (np.random.default_rng(seed + 1).random((n, 4, B, H)) >= rate).astype(np.uint8)


def postnet_masks(layers, B, T, C, rate=0.5, seed=5339):
    """Postnet dropout keep bits (modules.py:496-497, tacotron_dropout_rate 0.5, training=True):
    [layers, B, T, C] uint8."""
    return (np.random.default_rng(seed + 2).random((layers, B, T, C)) >= rate).astype(np.uint8)


def enc_conv_masks(layers, B, T, C, rate=0.5, seed=5339):
    """Encoder-convolution dropout keep bits (modules.py:496-497 in EncoderConvolutions,
    tacotron_dropout_rate 0.5, training=True): [layers, B, T, C] uint8."""
    return (np.random.default_rng(seed + 3).random((layers, B, T, C)) >= rate).astype(np.uint8)


def enc_zoneout_masks(T, B, U, rate=0.1, seed=5339):
    """Encoder BiLSTM training-zoneout keep bits by recurrence step (modules.py:236-240):
    [T, 2 (fw, bw), 2 (c, h), B, U] uint8."""
    return (np.random.default_rng(seed + 4).random((T, 2, 2, B, U)) >= rate).astype(np.uint8)
