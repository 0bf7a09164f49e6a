"""Tacotron_emt_attn host side (no GPU): weight key space and the oracle's structural properties.

GPU parity of the variant is tests/test_gpu_emt_attn.py."""
import numpy as np
import pytest

from _common import full_hparams, oracle_hp, prenet_masks, small_hparams, tacotron_inputs
from oracle import tacotron_emt_ref as ER


@pytest.mark.parametrize("attn,extra", [("simple", 128 + 128), ("multihead", 128),
                                        ("style_tokens", 64)])
def test_lstm1_rows(attn, extra):
    """LSTM-1 input = [prenet 256 | encoder context 512 | emotion block] (Architecture_wrappers.py:
    202-211) + the recurrent h rows."""
    from tt2.weights import tacotron_emt_weight_specs
    hp = full_hparams()
    rg = "gru_multi" if attn == "simple" else "none"
    S = dict((n, s) for n, s, _ in tacotron_emt_weight_specs(hp, attn, rg))
    k = S["Tacotron_model/inference/decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel"]
    assert k == (256 + 512 + extra + 1024, 4096)
    # memory = encoder outputs only (tacotron_emt_attn.py:244-246)
    assert S["Tacotron_model/inference/memory_layer/kernel"] == (512, 128)
    assert not any("style_tokens_" in n or "Multihead-attention-emt" in n for n in S)


def test_value_widths():
    from tt2.weights import emt_value_width
    hp = full_hparams()
    assert emt_value_width(hp, "multihead", "none") == 256    # ceil(80/64) x 128 filters
    assert emt_value_width(hp, "multihead", "gru") == 256     # [fw | bw] x reference_depth 128
    assert emt_value_width(hp, "simple", "gru_multi") == 128  # = attention_dim: 'simple' is buildable
    assert emt_value_width(hp, "style_tokens", "none") == 16


def _w(attn, rg, hp=None):
    from tt2.weights import init_tacotron_emt_weights
    hp = hp or small_hparams()
    return hp, init_tacotron_emt_weights(hp, attn, rg)


def test_bidirectional_gru_reverse_is_time_reversed_forward():
    """bidirectional_dynamic_rnn without lengths: the bw outputs are the bw cell run forward over
    the reversed sequence, then reversed back."""
    hp, W = _w("multihead", "gru")
    x = np.random.default_rng(0).normal(0, 1, (2, 6, 64)).astype(np.float32)
    s = "refnet_emt/bidirectional_rnn/bw/gru_cell/"
    bw = ER._gru_run(x, W, s, np.float32, reverse=True)
    fw_on_rev = ER._gru_run(x[:, ::-1].copy(), W, s, np.float32)
    np.testing.assert_array_equal(bw, fw_on_rev[:, ::-1])


@pytest.mark.parametrize("attn,rg", [("simple", "gru"), ("multihead", "none"),
                                     ("multihead", "gru_multi"), ("style_tokens", "none")])
def test_emotion_attention_weights_are_distributions(attn, rg):
    hp = small_hparams()
    if attn == "simple":
        hp.override_from_dict(dict(reference_depth=16))
    hp, W = _w(attn, rg, hp)
    ids, lens, re, rs = tacotron_inputs(2, 7, 200, seed=3)
    ev = ER.emotion_values(re, W, attn, rg)
    q = np.random.default_rng(1).normal(0, 1, (2, hp.decoder_lstm_units)).astype(np.float32)
    ctx, a = ER.emotion_attention(q, ev, W, attn, labels=[1, 2])
    np.testing.assert_allclose(a.sum(-1), 1.0, atol=1e-6)
    assert ctx.shape[-1] == ER.emt_state_width(W, attn)


def test_style_tokens_out_of_range_label_is_zero_row():
    """tf.one_hot(label >= depth) is all zeros: the query gets no label row."""
    hp, W = _w("style_tokens", "none")
    ev = ER.emotion_values(None, W, "style_tokens", "none")
    q = np.random.default_rng(2).normal(0, 1, (1, hp.decoder_lstm_units)).astype(np.float32)
    c_bad, _ = ER.emotion_attention(q, ev, W, "style_tokens", labels=[9], n_emt=4)
    Wz = dict(W)
    key = "Tacotron_model/inference/decoder/Multihead-attention-attn_emt/conv1d/kernel"
    Wz[key] = W[key].copy()
    Wz[key][0, hp.decoder_lstm_units:] = 0   # no label rows at all
    c_zero, _ = ER.emotion_attention(q, ev, Wz, "style_tokens", labels=[0], n_emt=4)
    np.testing.assert_allclose(c_bad, c_zero, atol=1e-7)


def test_synthesize_shapes():
    hp, W = _w("multihead", "gru_multi")
    ids, lens, re, rs = tacotron_inputs(2, 7, 200, seed=4)
    m = prenet_masks(6, 2, hp.prenet_layers[0], seed=4)
    r = ER.synthesize(ids, lens, re, rs, W, oracle_hp(hp), "multihead", "gru_multi", m, 6)
    assert r["alignments_emt"].shape == (r["frames"].shape[1], 2, hp.num_heads, 8)
    assert r["encoder_outputs"].shape[-1] == 2 * hp.encoder_lstm_units
