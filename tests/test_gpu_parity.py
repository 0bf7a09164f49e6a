"""GPU parity: libtt2.so (HIP, gfx950) vs the numpy oracle on identical seeded inputs.

Tolerances (BASELINE.json north_star): mel frames within 1e-4; MoL mixture indices bit-exact given
injected uniforms.  Intermediate tensors use the same 1e-4 absolute bound unless noted.
"""
import numpy as np
import pytest

from _common import (full_hparams, mol_uniforms, oracle_hp, prenet_masks, small_hparams,
                     small_wavenet_hparams, tacotron_inputs, wavenet_oracle_hp)
from oracle import tacotron_ref as TR
from oracle import wavenet_ref as WR

pytestmark = pytest.mark.gpu

MEL_TOL = 1e-4


def _engine(hp, W, B, T, T_ref, max_iters, constraint=False):
    from tt2.engine import TacotronEngine
    return TacotronEngine(hp, W, B, T, T_ref, max_iters, 0, False, constraint)


@pytest.fixture(scope="module")
def small_setup():
    from tt2.weights import init_tacotron_weights
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    return hp, W


@pytest.fixture(scope="module")
def full_setup():
    from tt2.weights import init_tacotron_weights
    hp = full_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    return hp, W


def test_library_loads_native():
    from tt2 import _lib
    lib = _lib.load_library()
    assert b"gfx950" in lib.tt2_version()


def test_mol_sampler_bit_exact():
    from tt2.engine import mol_sample
    rng = np.random.default_rng(0)
    n, nr = 4096, 10
    logits = rng.normal(0, 2, (n, 3 * nr)).astype(np.float32)
    # adversarial near-ties: duplicate logits on some rows
    logits[:256, 1] = logits[:256, 0]
    um = rng.uniform(1e-5, 1 - 1e-5, (n, nr)).astype(np.float32)
    um[:128, 1] = um[:128, 0]  # exact tie of (logit, uniform) -> first index wins
    ul = rng.uniform(1e-5, 1 - 1e-5, (n,)).astype(np.float32)
    lsm = float(np.log(1e-14))
    x, k = mol_sample(logits, um, ul, lsm)
    xr, kr = WR.mol_sample(logits, um, ul, lsm)
    np.testing.assert_array_equal(k, kr)
    np.testing.assert_allclose(x, xr, atol=2e-6, rtol=1e-5)


def test_mixture_shim_shapes():
    from wavenet_vocoder.models.mixture import sample_with_index
    rng = np.random.default_rng(1)
    y = rng.normal(0, 1, (2, 30, 17)).astype(np.float32)
    um = rng.uniform(1e-5, 1 - 1e-5, (2, 17, 10))
    ul = rng.uniform(1e-5, 1 - 1e-5, (2, 17))
    x, k = sample_with_index(y, -32.0, um, ul)
    xr, kr = WR.mol_sample(y.transpose(0, 2, 1).reshape(-1, 30), um.reshape(-1, 10),
                           ul.reshape(-1), -32.0)
    assert x.shape == (2, 17)
    np.testing.assert_array_equal(k.reshape(-1), kr)
    np.testing.assert_allclose(x.reshape(-1), xr, atol=2e-6)


@pytest.mark.parametrize("B,T", [(3, 11), (1, 5)])
def test_encoder_memory_small(small_setup, B, T):
    hp, W = small_setup
    ids, lens, re, rs = tacotron_inputs(B, T, 70, seed=7)
    eng = _engine(hp, W, B, T, 70, 8)
    mem, style = eng.encode(ids, lens, re, rs)
    oh = oracle_hp(hp)
    enc = TR.encoder(ids, lens, W, oh)
    st = TR.style_embedding(re, rs, W, oh)
    vals, _ = TR.memory_and_keys(enc, st, lens, W)
    np.testing.assert_allclose(style, st, atol=1e-5)
    np.testing.assert_allclose(mem, vals, atol=1e-5)
    eng.close()


def _decode_compare(hp, W, B, T, T_ref, n, targets=None, seed=11, constraint=False, tol=MEL_TOL):
    ids, lens, re, rs = tacotron_inputs(B, T, T_ref, seed=seed)
    P = hp.prenet_layers[0]
    masks = prenet_masks(n, B, P, seed=seed)
    eng = _engine(hp, W, B, T, T_ref, n, constraint)
    out = eng.synthesize(ids, lens, re, rs, n, masks, 0, targets)
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp, constraint), masks, n, targets)
    assert out["frames"].shape == ref["decoder_output"].shape
    np.testing.assert_allclose(out["stop_token_prediction"], ref["stop_token_prediction"], atol=tol)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], atol=tol)
    np.testing.assert_allclose(out["decoder_output"], ref["decoder_output"], atol=tol)
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], atol=tol)
    eng.close()
    return out, ref


def test_decoder_free_run_small(small_setup):
    hp, W = small_setup
    _decode_compare(hp, W, B=4, T=13, T_ref=64, n=30)


def test_decoder_window_constraint_small(small_setup):
    hp, W = small_setup
    _decode_compare(hp, W, B=2, T=17, T_ref=64, n=20, constraint=True)


def test_decoder_gta_small(small_setup):
    hp, W = small_setup
    B, n = 3, 60
    tg = np.random.default_rng(3).uniform(-4, 4, (B, 45, hp.num_mels)).astype(np.float32)
    out, ref = _decode_compare(hp, W, B=B, T=9, T_ref=64, n=n, targets=tg)
    assert out["frames"].shape[1] == 45  # TacoTrainingHelper stops at T_targets


def test_stop_rule_small(small_setup):
    """Batch-level stop (helpers.py:40-54): all rows stop together at the first step where every
    row rounds to 1; with a large positive stop bias that is step 0 -> 1 frame."""
    hp, W = small_setup
    W2 = dict(W)
    key = "Tacotron_model/inference/decoder/stop_token_projection/projection_stop_token_projection/bias"
    W2[key] = np.array([8.0], np.float32)
    out, ref = _decode_compare(hp, W2, B=3, T=7, T_ref=64, n=25)
    assert out["frames"].shape[1] == 1 == ref["decoder_output"].shape[1]


def test_stop_rule_mid_sequence(small_setup):
    """A stop bias near the decision boundary stops at an intermediate step; GPU and oracle must
    agree on the step (the stop probabilities themselves are compared at 1e-4)."""
    hp, W = small_setup
    W2 = dict(W)
    key = "Tacotron_model/inference/decoder/stop_token_projection/projection_stop_token_projection/bias"
    for bias in (0.6, 1.0, 1.5):
        W2[key] = np.array([bias], np.float32)
        out, ref = _decode_compare(hp, W2, B=2, T=7, T_ref=64, n=40, seed=5)
        assert out["frames"].shape[1] == ref["decoder_output"].shape[1]


def test_postnet_standalone(small_setup):
    hp, W = small_setup
    rng = np.random.default_rng(4)
    frames = rng.uniform(-5, 5, (2, 37, hp.num_mels)).astype(np.float32)
    eng = _engine(hp, W, 2, 8, 64, 40)
    dec, mel = eng.postnet(frames)
    rd, rm = TR.postnet_and_clip(frames, W, oracle_hp(hp))
    np.testing.assert_allclose(dec, rd, atol=1e-6)
    np.testing.assert_allclose(mel, rm, atol=MEL_TOL)
    eng.close()


@pytest.mark.parametrize("B,T", [(4, 150), (3, 1), (5, 61)])
def test_postnet_planes_path_full_dims(full_setup, monkeypatch, B, T):
    """512-channel Postnet over pre-split padded planes (gemm.h conv_x3) against the
    oracle and against the im2col GEMM path (TT2_POSTNET_CX=0); T=1 and B·(T+4) not a multiple of
    the 128-row tile cover the pad / guard rows."""
    hp, W = full_setup
    rng = np.random.default_rng(40 + T)
    frames = rng.uniform(-5, 5, (B, T, hp.num_mels)).astype(np.float32)
    outs = {}
    for cx, wide in (("1", "1"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("TT2_POSTNET_CX", cx)
        monkeypatch.setenv("TT2_CX_WIDE", wide)
        eng = _engine(hp, W, B, 8, 64, T)
        outs[cx + wide] = eng.postnet(frames)
        eng.close()
    rd, rm = TR.postnet_and_clip(frames, W, oracle_hp(hp))
    for k in ("11", "10"):  # 256 x 256 LDS-DMA kernel, 128 x 128 register-staged kernel
        np.testing.assert_allclose(outs[k][0], rd, atol=1e-6)
        np.testing.assert_allclose(outs[k][1], rm, atol=MEL_TOL)
    # same split, same k-step order (chunk-major, tap-minor): the planes kernels agree bit for bit;
    # the im2col path sums the same products in tap-major order
    np.testing.assert_array_equal(outs["11"][1], outs["10"][1])
    np.testing.assert_allclose(outs["11"][1], outs["01"][1], atol=1e-5)


@pytest.mark.parametrize("split", ["4", "1", "7"])
def test_encoder_planes_path_full_dims(full_setup, monkeypatch, split):
    """Text encoder on the planes path (3 convs with K split over work-groups + the BiLSTM input
    projection as a width-1 conv) at configs[1]'s B=32 x 201 ragged, against the
    oracle and the im2col GEMM path (TT2_ENC_CX=0)."""
    hp, W = full_setup
    B, T = 32, 201
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=21)
    monkeypatch.setenv("TT2_ENC_SPLITK", split)
    outs = {}
    for cx in ("1", "0"):
        monkeypatch.setenv("TT2_ENC_CX", cx)
        eng = _engine(hp, W, B, T, 64, 4)
        outs[cx] = eng.encode(ids, lens, re, rs)
        eng.close()
    oh = oracle_hp(hp)
    enc = TR.encoder(ids, lens, W, oh)
    st = TR.style_embedding(re, rs, W, oh)
    vals, _ = TR.memory_and_keys(enc, st, lens, W)
    np.testing.assert_allclose(outs["1"][0], vals, atol=1e-4)
    np.testing.assert_allclose(outs["1"][0], outs["0"][0], atol=2e-5)


def test_full_dims_free_run(full_setup):
    """Fork-default dimensions (D_mem 1024, 2x1024 LSTM, 512-ch postnet), short horizon."""
    hp, W = full_setup
    _decode_compare(hp, W, B=4, T=23, T_ref=96, n=12)


def test_full_dims_gta(full_setup):
    hp, W = full_setup
    B = 2
    tg = np.random.default_rng(9).uniform(-4, 4, (B, 40, hp.num_mels)).astype(np.float32)
    _decode_compare(hp, W, B=B, T=15, T_ref=64, n=40, targets=tg)


# ---- persistent decoder (k_decode_persist: one launch, weights resident on-chip) ----

def _persistent(eng):
    return eng.decoder_path()[0] == 1


def test_persistent_full_batch_free_run(full_setup):
    """configs[1] shape (B=32, 200 chars + EOS, ragged lengths) through the persistent decoder,
    free running with injected prenet masks, against the oracle over 50 steps."""
    hp, W = full_setup
    out, ref = _decode_compare(hp, W, B=32, T=201, T_ref=96, n=50, seed=21)


def test_trained_refnet_weights_persistent(full_setup):
    """The reference's own trained emotion reference encoder (refnet_emt, ckpt-5200, restored
    the way tacotron/train.py:284 does; committed as tests/golden/refnet_emt_ckpt5200.npz) in
    place of the random refnet_emt weights: encoder + style path + persistent decoder vs oracle."""
    import os
    hp, W = full_setup
    fx = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "refnet_emt_ckpt5200.npz")
    W2 = dict(W)
    with np.load(fx) as z:
        for k in z.files:
            assert W2[k].shape == z[k].shape, k
            W2[k] = z[k]
    _decode_compare(hp, W2, B=32, T=121, T_ref=96, n=30, seed=31)


def test_persistent_selected_for_bench_shape(full_setup):
    hp, W = full_setup
    ids, lens, re, rs = tacotron_inputs(32, 201, 64, seed=4)
    eng = _engine(hp, W, 32, 201, 64, 4)
    eng.synthesize(ids, lens, re, rs, 4, prenet_masks(4, 32, hp.prenet_layers[0], seed=4))
    assert _persistent(eng), "k_decode_persist not used at configs[1] shapes on this device"
    eng.close()


def test_persistent_partial_batch_window(full_setup):
    """Padding rows (B=5 < 32) and the synthesis window constraint (attention.py:202-215)."""
    hp, W = full_setup
    _decode_compare(hp, W, B=5, T=57, T_ref=64, n=30, seed=8, constraint=True)


def test_persistent_gta_full_batch(full_setup):
    hp, W = full_setup
    B = 32
    tg = np.random.default_rng(12).uniform(-4, 4, (B, 33, hp.num_mels)).astype(np.float32)
    out, ref = _decode_compare(hp, W, B=B, T=120, T_ref=64, n=40, targets=tg, seed=12)
    assert out["frames"].shape[1] == 33


def test_persistent_stop_rule(full_setup):
    """Batch-level stop decided from the flags' stop bits: GPU and oracle stop at the same step."""
    hp, W = full_setup
    W2 = dict(W)
    key = "Tacotron_model/inference/decoder/stop_token_projection/projection_stop_token_projection/bias"
    for bias in (0.3, 0.8, 8.0):
        W2[key] = np.array([bias], np.float32)
        out, ref = _decode_compare(hp, W2, B=6, T=31, T_ref=64, n=40, seed=6)
        assert out["frames"].shape[1] == ref["decoder_output"].shape[1]


def test_persistent_repeat_calls_after_early_stop(full_setup):
    """Granule tags restart every launch: a decode that stopped after 2 steps must not leave tags
    that a second decode on the same context accepts as fresh."""
    hp, W = full_setup
    B, T, n = 4, 19, 20
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=17)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=17)
    eng = _engine(hp, W, B, T, 64, n)
    ids0, lens0, re0, rs0 = tacotron_inputs(B, T, 64, seed=99)  # different first call
    first = eng.synthesize(ids0, lens0, re0, rs0, 2, prenet_masks(2, B, hp.prenet_layers[0], seed=99))
    assert first["frames"].shape[1] == 2
    again = eng.synthesize(ids, lens, re, rs, n, masks)      # same context, full horizon
    eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    np.testing.assert_allclose(again["decoder_output"], ref["decoder_output"], atol=MEL_TOL)
    np.testing.assert_allclose(again["alignments"], ref["alignments"], atol=MEL_TOL)


@pytest.mark.parametrize("B,T,n,constraint", [(8, 300, 30, False), (3, 512, 20, True), (32, 257, 12, False)])
def test_persistent_long_inputs_match_oracle(full_setup, B, T, n, constraint):
    """T_in > 256 on the persistent decoder (k_decode_persist<false, 512>: values of positions
    [256, T_in) streamed per step, cumulative alignments over 512 + 31 taps): ragged rows, the
    window constraint at T_in = 512, and the 257 boundary with a full 32-row batch, against the
    oracle (attention.py:170-227 has no length cliff)."""
    hp, W = full_setup
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=T)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=T)
    eng = _engine(hp, W, B, T, 64, n, constraint)
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    assert _persistent(eng), "k_decode_persist not used at T_in = %d" % T
    eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp, constraint), masks, n)
    assert int(lens.max()) > 256
    assert out["frames"].shape == ref["decoder_output"].shape
    np.testing.assert_allclose(out["stop_token_prediction"], ref["stop_token_prediction"], atol=MEL_TOL)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], atol=MEL_TOL)
    np.testing.assert_allclose(out["decoder_output"], ref["decoder_output"], atol=MEL_TOL)
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], atol=MEL_TOL)


def test_persistent_long_inputs_match_launch_path(full_setup):
    """T_in = 300 over 400 steps: the long-input persistent decoder against the per-step launch
    path (the attention walks past position 256 within the horizon)."""
    import os
    hp, W = full_setup
    B, T, n = 32, 300, 400
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=77)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=77)
    eng = _engine(hp, W, B, T, 64, n)
    a = eng.synthesize(ids, lens, re, rs, n, masks)
    assert _persistent(eng)
    a = eng.synthesize(ids, lens, re, rs, n, masks)  # timed second launch
    print("T_in=%d persistent decoder: %.2f us/step" % (T, 1e3 * eng.decoder_path()[1] / a["frames"].shape[1]))
    eng.close()
    os.environ["TT2_DECODER"] = "launch"
    try:
        eng2 = _engine(hp, W, B, T, 64, n)
    finally:
        del os.environ["TT2_DECODER"]
    b = eng2.synthesize(ids, lens, re, rs, n, masks)
    assert not _persistent(eng2)
    eng2.close()
    assert a["frames"].shape == b["frames"].shape
    np.testing.assert_allclose(a["stop_token_prediction"], b["stop_token_prediction"], atol=1e-4)
    np.testing.assert_allclose(a["alignments"], b["alignments"], atol=1e-4)
    np.testing.assert_allclose(a["decoder_output"], b["decoder_output"], atol=1e-4)


def test_persistent_matches_launch_path_long(full_setup):
    """1000-step horizon at configs[1] shapes: persistent decoder vs the per-step launch path
    (both HIP; the oracle is too slow for 1000 steps x 32 rows in a unit test)."""
    import os
    hp, W = full_setup
    B, T, n = 32, 201, 1000
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=31)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=31)
    eng = _engine(hp, W, B, T, 64, n)
    a = eng.synthesize(ids, lens, re, rs, n, masks)
    assert _persistent(eng)
    eng.close()
    os.environ["TT2_DECODER"] = "launch"
    try:
        eng2 = _engine(hp, W, B, T, 64, n)
    finally:
        del os.environ["TT2_DECODER"]
    b = eng2.synthesize(ids, lens, re, rs, n, masks)
    assert not _persistent(eng2)
    eng2.close()
    assert a["frames"].shape == b["frames"].shape
    np.testing.assert_allclose(a["stop_token_prediction"], b["stop_token_prediction"], atol=1e-4)
    np.testing.assert_allclose(a["alignments"], b["alignments"], atol=1e-4)
    np.testing.assert_allclose(a["decoder_output"], b["decoder_output"], atol=1e-4)


def test_tacotron_shim_initialize(small_setup):
    """tacotron.models.create_model('Tacotron', hp).initialize(...) fills tower_* like the
    reference (tacotron.py:573-632)."""
    from types import SimpleNamespace

    from tacotron.models import create_model
    hp, W = small_setup
    hp = hp.copy()
    hp.max_iters = 15
    B, T = 2, 9
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=2)
    masks = prenet_masks(15, B, hp.prenet_layers[0], seed=2)
    m = create_model("Tacotron", hp)
    m.load_weights(W)
    args = SimpleNamespace(emt_only=False, adain=False, unpaired=False, nat_gan=False,
                           pretrained_emb_disc_all=False, synth_constraint=False)
    m.initialize(args, ids, lens, ref_mel_emt=re, ref_mel_spk=rs, n_emt=4, n_spk=2, synth=True,
                 prenet_masks=masks)
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, 15)
    assert len(m.tower_mel_outputs) == 1
    np.testing.assert_allclose(m.tower_mel_outputs[0], ref["mel_outputs"], atol=MEL_TOL)
    assert m.tower_alignments[0].shape == ref["alignments"].shape


# ------------------------------------------------------------------------------------ WaveNet

def _wn(hp, W, maxB, maxT):
    from tt2.engine import WaveNetEngine
    return WaveNetEngine(hp, W, maxB, maxT, 0)


@pytest.mark.parametrize("layers,stacks,B,T_f", [(6, 2, 2, 2), (24, 4, 2, 2), (24, 4, 20, 1)])
def test_wavenet_teacher_forced(layers, stacks, B, T_f):
    """B = 20: the reference's batched synthesis (wavenet_synthesis_batch_size, hparams.py:332), all
    rows in one generation launch of k_generate_pipe."""
    from tt2.weights import init_wavenet_weights
    hp = small_wavenet_hparams(layers, stacks)
    W = init_wavenet_weights(hp, seed=5339)
    rng = np.random.default_rng(21)
    T = T_f * 275
    mel = rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32)
    cond = WR.interp_condition(mel)
    um, ul = mol_uniforms(T, B, seed=3)
    teacher = rng.uniform(-0.9, 0.9, (B, T)).astype(np.float32)
    eng = _wn(hp, W, B, T)
    out = eng.generate(cond, um, ul, 0, teacher, want_logits=True, want_upsampled=True)
    c_up = WR.upsample_2d(cond.transpose(0, 2, 1), W, hp.upsample_scales)
    np.testing.assert_allclose(out["upsampled"], c_up, atol=1e-5)
    y, k, lg = WR.incremental(c_up.transpose(0, 2, 1), W, wavenet_oracle_hp(hp), um, ul, teacher,
                              return_logits=True)
    np.testing.assert_allclose(out["logits"], lg, atol=1e-4, rtol=1e-4)
    # bit-exact mixture indices unless the oracle's own Gumbel margin is below fp32 resolution
    gl = np.log(-np.log(um.astype(np.float64))).astype(np.float32)
    temp = lg[..., :10] - gl.transpose(1, 0, 2)
    srt = np.sort(temp, -1)
    margin = srt[..., -1] - srt[..., -2]
    safe = margin > 1e-4
    assert safe.mean() > 0.99
    np.testing.assert_array_equal(out["k"][safe], k[safe])
    np.testing.assert_allclose(out["y"][safe], y[safe], atol=1e-4)
    eng.close()


def test_wavenet_free_run_short():
    from tt2.weights import init_wavenet_weights
    hp = small_wavenet_hparams(24, 4)
    W = init_wavenet_weights(hp, seed=5339)
    rng = np.random.default_rng(5)
    B, T_f = 1, 1
    T = 275
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32))
    um, ul = mol_uniforms(T, B, seed=8)
    out = _wn(hp, W, B, T).generate(cond, um, ul, 0, None)
    c_up = WR.upsample_2d(cond.transpose(0, 2, 1), W, hp.upsample_scales)
    y, k = WR.incremental(c_up.transpose(0, 2, 1), W, wavenet_oracle_hp(hp), um, ul)
    # free running: identical until a (rare) near-tie diverges; require a long identical prefix
    same = out["k"][0] == k[0]
    first_diff = int(np.argmin(same)) if not same.all() else T
    assert first_diff >= 200
    np.testing.assert_allclose(out["y"][0, :first_diff], y[0, :first_diff], atol=1e-4)


def test_wavenet_shim_initialize():
    from wavenet_vocoder.models import create_model
    hp = small_wavenet_hparams(6, 2)
    m = create_model("WaveNet", hp)
    m.init_random_weights()
    rng = np.random.default_rng(6)
    c = WR.interp_condition(rng.uniform(-4, 4, (2, 1, 80)).astype(np.float32))
    um, ul = mol_uniforms(275, 2, seed=1)
    m.initialize(None, c, None, None, u_mix=um, u_log=ul)
    assert m.tower_y_hat[0].shape == (2, 275)
    assert m.tower_synth_upsampled_local_features[0].shape == (2, 80, 275)
    assert np.all(np.abs(m.tower_y_hat[0]) <= 1.0)


def test_wavenet_shim_mulaw_input_type():
    """input_type='mulaw' (wavenet.py:459-460): the same scalar-input generation as 'raw' (start
    silence mulaw(0.0) = 0), the companded samples expanded with inv_mulaw (mu = 255) at the end."""
    from wavenet_vocoder.models import create_model
    from wavenet_vocoder.util import inv_mulaw
    rng = np.random.default_rng(6)
    c = WR.interp_condition(rng.uniform(-4, 4, (2, 1, 80)).astype(np.float32))
    um, ul = mol_uniforms(275, 2, seed=1)
    ys = {}
    for it in ("raw", "mulaw"):
        hp = small_wavenet_hparams(6, 2)
        hp.override_from_dict(dict(input_type=it))
        m = create_model("WaveNet", hp)
        m.init_random_weights()
        m.initialize(None, c, None, None, u_mix=um, u_log=ul)
        ys[it] = m.tower_y_hat[0]
    np.testing.assert_allclose(ys["mulaw"], inv_mulaw(ys["raw"]).astype(np.float32), rtol=1e-6, atol=1e-7)
    assert np.abs(ys["mulaw"]).max() < np.abs(ys["raw"]).max() + 1e-6


# ----------------------------------------------------------- single-step seam (tt2_decoder_step)

def test_decoder_step_golden_fixture(full_setup):
    """tt2_decoder_step (TacotronDecoderCell.__call__, Architecture_wrappers.py:197-267) from the
    committed fixture's non-trivial state: every output and next-state array vs the oracle's."""
    import os
    hp, W = full_setup
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             "tacotron_decoder_step.npz"))
    ids, lens = g["ids"], g["lengths"]
    eng = _engine(hp, W, ids.shape[0], ids.shape[1], g["ref_emt"].shape[1], 4)
    eng.encode(ids, lens, g["ref_emt"], g["ref_spk"])
    names = ("h1", "c1", "h2", "c2", "attention", "alignments", "max_attentions")
    state = {k: g["in_" + k] for k in names}
    state["time"] = 5
    frame, stop, align, nxt = eng.decoder_step(g["frame_in"], g["prenet_masks"], state)
    eng.close()
    np.testing.assert_allclose(frame, g["frame"], atol=1e-5)
    np.testing.assert_allclose(stop, g["stop"], atol=1e-6)
    np.testing.assert_allclose(align, g["align"], atol=1e-6)
    for k in names[:-1]:
        np.testing.assert_allclose(nxt[k], g["out_" + k], atol=1e-5, err_msg=k)
    np.testing.assert_array_equal(nxt["max_attentions"], g["out_max_attentions"])
    assert nxt["time"] == 6


@pytest.mark.parametrize("constraint", [False, True])
def test_decoder_step_chain_matches_decode(small_setup, constraint):
    """Driving tt2_decoder_step from zero_state with the previous raw frame as input (TacoTestHelper,
    helpers.py:57) reproduces tt2_decode's fused loop step for step."""
    hp, W = small_setup
    B, T, n = 3, 11, 12
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=13)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=13)
    eng = _engine(hp, W, B, T, 64, n, constraint)
    full = eng.synthesize(ids, lens, re, rs, n, masks)
    eng.encode(ids, lens, re, rs)
    state = eng.zero_state()
    frame = np.zeros((B, hp.num_mels), np.float32)
    for t in range(full["frames"].shape[1]):
        frame, stop, align, state = eng.decoder_step(frame, masks[t], state)
        np.testing.assert_allclose(frame, full["frames"][:, t], atol=1e-5)
        np.testing.assert_allclose(stop, full["stop_token_prediction"][:, t], atol=1e-5)
        np.testing.assert_allclose(align, full["alignments"][:, :, t], atol=1e-5)
    eng.close()


def test_cpu_backend_noise_streams_match_device():
    """libtt2_cpu.so and libtt2.so draw identical seeded prenet keep bits and MoL uniforms (one
    rng.h): the CPU baseline runs exactly the GPU bench's workload."""
    import os
    import subprocess
    from tt2 import _lib
    from tt2.engine import prenet_keep_bits, wavenet_noise
    if not os.path.exists(_lib.CPU_LIB_PATH):
        subprocess.check_call(["make", "-C", os.path.dirname(_lib.CPU_LIB_PATH), "libtt2_cpu.so"])
    cpu = _lib.load_cpu_library()
    n, B, P = 7, 3, 256
    bits = np.zeros((n, 2, B, P), np.uint8)
    _lib.check(cpu.tt2_prenet_keep_bits(5339, n, B, P, _lib.ptr(bits)), cpu)
    np.testing.assert_array_equal(bits, prenet_keep_bits(5339, n, B, P))
    T = 50
    um = np.zeros((T, B, 10), np.float32)
    ul = np.zeros((T, B), np.float32)
    _lib.check(cpu.tt2_wn_noise(91, T, B, 10, 0, _lib.ptr(um), _lib.ptr(ul)), cpu)
    gm, gl = wavenet_noise(91, T, B, 10)
    np.testing.assert_array_equal(um, gm)
    np.testing.assert_array_equal(ul, gl)


@pytest.mark.parametrize("widths", ["small", "fork"])
def test_smoothing_normalization(widths):
    """hp.smoothing (attention.py:71-80,150): sigmoid normalisation on the launch path (the
    persistent decoder is never chosen for it), free running, within 1e-4 of the oracle; a chain of
    tt2_decoder_step calls (the step seam's own kernels) reproduces the fused loop."""
    from tt2.weights import init_tacotron_weights
    hp = small_hparams() if widths == "small" else full_hparams()
    hp.override_from_dict(dict(smoothing=True))
    W = init_tacotron_weights(hp, seed=5339)
    B, T, n = 3, 23, 12
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=72)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=72)
    eng = _engine(hp, W, B, T, 40, n)
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    assert eng.decoder_path()[0] == 0
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], rtol=0, atol=MEL_TOL)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], rtol=0, atol=1e-4)
    eng.encode(ids, lens, re, rs)
    state = eng.zero_state()
    frame = np.zeros((B, hp.num_mels), np.float32)
    for t in range(out["frames"].shape[1]):
        frame, stop, align, state = eng.decoder_step(frame, masks[t], state)
        np.testing.assert_allclose(align, out["alignments"][:, :, t], atol=1e-5)
        np.testing.assert_allclose(frame, out["frames"][:, t], atol=1e-5)
    eng.close()


@pytest.mark.parametrize("stop_at_any,bias,scale,steps", [(False, -6.0, 1, 14), (True, -3.0, 30, 14),
                                                         (True, 4.0, 1, 1)])
def test_chunked_tower_b48_matches_oracle(stop_at_any, bias, scale, steps):
    """A 48-row tower (two 24-row contexts decoding without their own stop rule, the tower's stop
    step taken over all rows afterwards) against one oracle decode of all 48 rows (VERDICT r04
    item 7; hparams.py:44 batches up to 96 rows per tower)."""
    from _common import STOP_BIAS
    from tt2.weights import init_tacotron_weights
    hp = small_hparams()
    hp.override_from_dict(dict(stop_at_any=stop_at_any))
    W = init_tacotron_weights(hp, seed=5339)
    W[STOP_BIAS] = np.full((1,), bias, np.float32)
    K = STOP_BIAS.replace("/bias", "/kernel")
    W[K] = W[K] * scale
    B, T, n = 48, 11, 14
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=23)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=23)
    eng = _engine(hp, W, B, T, 40, n)
    assert [c.caps[0] for c in eng._chunks] == [24, 24]
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    if steps is not None:
        assert ref["mel_outputs"].shape[1] == steps
    else:
        assert 1 < ref["mel_outputs"].shape[1] < n
    assert out["mel_outputs"].shape == ref["mel_outputs"].shape
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], rtol=0, atol=MEL_TOL)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], rtol=0, atol=1e-5)
