"""Tacotron_emt_attn (tacotron_emt_attn.py): libtt2.so vs
oracle/tacotron_emt_ref.py on identical seeded inputs and injected prenet masks -- on the launch-path
decoder, and ('multihead' at the fork widths, round 3) in the persistent decoder.

Each emotion-attention type the reference builds ('simple', 'multihead', 'style_tokens') with the
reference-encoder output variants args.emt_ref_gru = 'none' / 'gru' / 'gru_multi', with and without
refnet_spk, free running and GTA.  Same 1e-4 bound as the Tacotron parity tests (test_gpu_parity);
the emotion attention weights of every step are compared too.  Parity unpinned: the reference
ships no checkpoint or fixture of this model (oracle/__init__.py).
"""
import numpy as np
import pytest

from _common import full_hparams, oracle_hp, prenet_masks, small_hparams, tacotron_inputs
from oracle import tacotron_emt_ref as ER

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _case(hp, attn, ref_gru, emt_only=False, B=3, T=11, T_ref=300, n=24, seed=21, targets=None,
          labels=None, n_emt=4, persistent_expected=0):
    from tt2.engine import TacotronEngine
    from tt2.weights import init_tacotron_emt_weights
    W = init_tacotron_emt_weights(hp, attn, ref_gru, emt_only, n_emt, seed=5339)
    ids, lens, re, rs = tacotron_inputs(B, T, T_ref, seed=seed)
    if attn == "style_tokens":
        re = rs = None
    elif emt_only:
        rs = None
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=seed)
    eng = TacotronEngine(hp, W, B, T, T_ref, n, 0, emt_only, False, attn, ref_gru, n_emt)
    if labels is not None:
        eng.set_emt_labels(labels)
    out = eng.synthesize(ids, lens, re, rs, n, masks, 0, targets)
    a_emt = eng.emt_alignments()
    persistent, _ = eng.decoder_path()
    eng.close()
    ref = ER.synthesize(ids, lens, re, rs, W, oracle_hp(hp), attn, ref_gru, masks, n, labels,
                        n_emt, emt_only, targets)
    assert persistent == persistent_expected
    assert out["frames"].shape == ref["decoder_output"].shape
    np.testing.assert_allclose(out["stop_token_prediction"], ref["stop_token_prediction"], atol=TOL)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], atol=TOL)
    np.testing.assert_allclose(out["decoder_output"], ref["decoder_output"], atol=TOL)
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], atol=TOL)
    # oracle [steps, B, heads, T_v] -> [B, heads, T_v, steps]
    np.testing.assert_allclose(a_emt, ref["alignments_emt"].transpose(1, 2, 3, 0), atol=TOL)
    return out, ref


def _small(**kw):
    hp = small_hparams()
    hp.override_from_dict(kw)
    return hp


def test_simple_gru():
    """'simple' needs the value width = attention_dim (the zero attention_emt state is
    attention_dim wide): reference_depth 16 -> [fw | bw] = 32 = attention_dim."""
    _case(_small(reference_depth=16), "simple", "gru")


def test_simple_gru_multi_full_width():
    """The only 'simple' combination at the fork's own widths: 8 x dense(128) = attention_dim; it
    decodes in the persistent decoder (round 5)."""
    _case(full_hparams(), "simple", "gru_multi", B=2, T=9, T_ref=80, n=12, persistent_expected=1)


@pytest.mark.parametrize("ref_gru", ["none", "gru", "gru_multi"])
def test_multihead(ref_gru):
    _case(small_hparams(), "multihead", ref_gru)


def test_multihead_emt_only_gta():
    hp = small_hparams()
    tg = np.random.default_rng(4).uniform(-4, 4, (2, 20, hp.num_mels)).astype(np.float32)
    out, _ = _case(hp, "multihead", "gru_multi", emt_only=True, B=2, n=30, targets=tg)
    assert out["frames"].shape[1] == 20


def test_style_tokens_labels():
    """One-hot emotion labels in the query; an out-of-range label is a zero row (tf.one_hot)."""
    _case(small_hparams(), "style_tokens", "none", B=4, labels=[0, 3, 1, 7])


def test_simple_rejects_inconsistent_width():
    """'simple' with values wider than attention_dim cannot be built by TF (the attention_emt
    state would change width); the library refuses it at create time."""
    from tt2.engine import TacotronEngine
    from tt2.weights import init_tacotron_emt_weights
    hp = small_hparams()
    W = init_tacotron_emt_weights(hp, "multihead", "none")
    with pytest.raises(RuntimeError, match="attention_dim"):
        TacotronEngine(hp, W, 2, 8, 64, 4, 0, False, False, "simple", "none")


def test_shim_initialize_and_synthesizer():
    """create_model('Tacotron_emt_attn') (models/__init__.py:8-9) + initialize with args.attn /
    args.emt_ref_gru, and the Synthesizer's emt_attn switch (synthesizer.py:24), against the
    oracle."""
    from types import SimpleNamespace
    from tacotron.models import create_model
    from tacotron.synthesizer import Synthesizer
    hp = small_hparams()
    hp.override_from_dict(dict(max_iters=16, tacotron_synthesis_batch_size=1))
    args = SimpleNamespace(attn="multihead", emt_ref_gru="gru", emt_only=False, emt_attn=True)
    m = create_model("Tacotron_emt_attn", hp)
    m.init_random_weights(attn="multihead", emt_ref_gru="gru")
    ids, lens, re, rs = tacotron_inputs(2, 9, 200, seed=31)
    masks = prenet_masks(16, 2, hp.prenet_layers[0], seed=31)
    m.initialize(args, ids, lens, ref_mel_emt=re, ref_mel_spk=rs, prenet_masks=masks, n_emt=4,
                 n_spk=2)
    ref = ER.synthesize(ids, lens, re, rs, m._weights, oracle_hp(hp), "multihead", "gru", masks, 16)
    np.testing.assert_allclose(m.tower_mel_outputs[0], ref["mel_outputs"], atol=TOL)
    syn = Synthesizer()
    syn.load(args, None, hp)
    mels = syn.synthesize(["hello there"], None, None, None, [None], mel_ref_filenames_emt=[re[0]],
                          mel_ref_filenames_spk=[rs[0]])
    assert len(mels) == 1 and mels[0].shape[1] == hp.num_mels and np.isfinite(mels[0]).all()


@pytest.mark.parametrize("ref_gru", ["gru", "gru_multi", "none"])
def test_multihead_full_width_persistent(ref_gru):
    """'multihead' at the fork widths runs in k_decode_persist<true>: the emotion query as 8 more
    projection tiles, 16 emotion work-groups (scores, softmax, heads-concatenated contexts), the
    attn_emt dense on the query blocks, the emotion block folded into the next step's LSTM-1 rows.
    heads x value width: 'gru' 4 x 256, 'gru_multi' 4 x 128, 'none' 4 x 256 (the CNN output)."""
    _case(full_hparams(), "multihead", ref_gru, B=3, T=9, T_ref=80, n=12, persistent_expected=1)


def test_multihead_full_width_persistent_emt_only_gta():
    """emt_only (no refnet_spk term) + GTA, padding rows of the 32-row tiles, persistent decoder."""
    hp = full_hparams()
    tg = np.random.default_rng(3).normal(0, 1, (2, 10, hp.num_mels)).astype(np.float32)
    _case(hp, "multihead", "gru_multi", emt_only=True, B=2, T=9, T_ref=80, n=14, targets=tg,
          persistent_expected=1)


@pytest.mark.parametrize("ref_gru", ["gru", "gru_multi"])
def test_multihead_persistent_configs1_gta_vs_oracle(ref_gru):
    """configs[1] shape (B = 32 ragged rows x 201 chars, T_ref 400) through k_decode_persist<true>,
    200 teacher-forced steps against the oracle at the north_star 1e-4: frames, stop tokens,
    alignments, mels and every step's emotion attention weights."""
    hp = full_hparams()
    B, T, TR, n = 32, 201, 400, 200
    tg = np.random.default_rng(3).normal(0, 1, (B, n, hp.num_mels)).astype(np.float32)
    out, _ = _case(hp, "multihead", ref_gru, B=B, T=T, T_ref=TR, n=n, seed=7, targets=tg,
                   persistent_expected=1)
    assert out["frames"].shape[1] == n


def test_multihead_persistent_matches_launch_path_b32():
    """configs[1]-shaped batch (B = 32, T_ref 400): persistent decoder against the launch path over
    80 free-running steps, same weights, inputs and prenet masks (split fp16x3 vs fp32 MFMA products:
    the two paths agree to float rounding, compared at 1e-3)."""
    import os
    from tt2.engine import TacotronEngine
    from tt2.weights import init_tacotron_emt_weights
    hp = full_hparams()
    B, T, TR, n = 32, 41, 400, 80
    W = init_tacotron_emt_weights(hp, "multihead", "gru", seed=5339)
    ids, lens, re, rs = tacotron_inputs(B, T, TR, seed=7)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=7)
    outs = []
    for mode in ("persistent", "launch"):
        old = os.environ.get("TT2_DECODER")
        os.environ["TT2_DECODER"] = mode
        try:
            eng = TacotronEngine(hp, W, B, T, TR, n, 0, False, False, "multihead", "gru", 4)
        finally:
            if old is None:
                del os.environ["TT2_DECODER"]
            else:
                os.environ["TT2_DECODER"] = old
        out = eng.synthesize(ids, lens, re, rs, n, masks)
        persistent, _ = eng.decoder_path()
        outs.append((out, eng.emt_alignments(), persistent))
        eng.close()
    (a, ea, pa), (b, eb, pb) = outs
    assert pa == 1 and pb == 0
    steps = min(a["frames"].shape[1], b["frames"].shape[1])
    assert steps >= 20
    np.testing.assert_allclose(a["frames"][:, :steps], b["frames"][:, :steps], atol=1e-3)
    np.testing.assert_allclose(ea[..., :steps], eb[..., :steps], atol=1e-3)


def test_style_tokens_full_width_persistent():
    """'style_tokens' at the fork widths runs in k_decode_persist<true> (round 5): the emotion query
    [h2 | one-hot label] as 8 more projection tiles (label rows in the per-row query bias), the 16
    emotion work-groups attend over the 24 shared tanh(style tokens) (4 heads x 16), and the
    heads-concatenated contexts are the 64-wide LSTM-1 block themselves (no dense, no speaker term).
    Ragged rows with an out-of-range label (tf.one_hot's zero row), against the oracle at 1e-4."""
    _case(full_hparams(), "style_tokens", "none", B=4, T=9, T_ref=80, n=14, labels=[0, 3, 1, 7],
          persistent_expected=1)


def test_style_tokens_persistent_configs1_gta_vs_oracle():
    """configs[1] shape (B = 32 ragged rows x 201 chars) through the persistent 'style_tokens'
    decoder, 200 teacher-forced steps against the oracle at 1e-4, every step's emotion weights too."""
    hp = full_hparams()
    B, T, n = 32, 201, 200
    tg = np.random.default_rng(5).normal(0, 1, (B, n, hp.num_mels)).astype(np.float32)
    labels = [i % 5 for i in range(B)]
    out, _ = _case(hp, "style_tokens", "none", B=B, T=T, T_ref=80, n=n, seed=9, targets=tg, labels=labels,
                   persistent_expected=1)
    assert out["frames"].shape[1] == n


def test_simple_full_width_persistent_emt_only_and_launch_path():
    """'simple' in k_decode_persist<true> (round 5): V(tanh(W1 v + W2 q)) over the 128 units as four
    32-unit partials summed into one softmax per row over the 8 'gru_multi' heads, the 128-wide context
    as the block's first half, refnet_spk's half folded into a per-row LSTM-1 bias; emt_only (no
    speaker half) too, and the launch path (TT2_DECODER=launch) on the same case."""
    import os
    _case(full_hparams(), "simple", "gru_multi", emt_only=True, B=3, T=9, T_ref=80, n=12, persistent_expected=1)
    os.environ["TT2_DECODER"] = "launch"
    try:
        _case(full_hparams(), "simple", "gru_multi", B=3, T=9, T_ref=80, n=12, persistent_expected=0)
    finally:
        del os.environ["TT2_DECODER"]


def test_simple_persistent_configs1_gta_vs_oracle():
    """configs[1] shape (B = 32 ragged rows x 201 chars, T_ref 400) through the persistent 'simple'
    decoder, 200 teacher-forced steps against the oracle at 1e-4, every step's emotion weights too."""
    hp = full_hparams()
    B, T, TR, n = 32, 201, 400, 200
    tg = np.random.default_rng(8).normal(0, 1, (B, n, hp.num_mels)).astype(np.float32)
    out, _ = _case(hp, "simple", "gru_multi", B=B, T=T, T_ref=TR, n=n, seed=11, targets=tg, persistent_expected=1)
    assert out["frames"].shape[1] == n
