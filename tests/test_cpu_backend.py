"""libtt2_cpu.so (tacotron-2_amd/cpu/tt2_cpu.cpp): the same C ABI on host cores — the timed CPU
baseline of bench.py and a second implementation of the path — against the committed golden
fixtures and the numpy oracle.  Runs without a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from _common import (full_hparams, mol_uniforms, oracle_hp, prenet_masks, small_hparams,
                     small_wavenet_hparams, tacotron_inputs, wavenet_oracle_hp)
from oracle import tacotron_ref as TR
from oracle import wavenet_ref as WR
from tt2 import _lib
from tt2.weights import init_tacotron_weights, init_wavenet_weights

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def cpu():
    if not os.path.exists(_lib.CPU_LIB_PATH):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "tacotron-2_amd"), "libtt2_cpu.so"])
    return _lib.load_cpu_library()


def _gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _taco(cpu, hp, W, B, T, T_ref, n, constraint=False):
    from tt2.engine import TacotronEngine
    return TacotronEngine(hp, W, B, T, T_ref, n, 0, False, constraint, lib=cpu)


def test_exports_are_header_symbols(cpu):
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.CPU_LIB_PATH]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip().startswith(("0", "T")) or
                   " T " in l)
    header = set(re.findall(r"\b(tt2_[a-z0-9_]+)\s*\(",
                            open(os.path.join(ROOT, "include", "tt2.h")).read()))
    tt2 = {s for s in exported if s.startswith("tt2_")}
    assert tt2 == set(_lib.CPU_SYMBOLS)
    assert tt2 <= header
    assert cpu.tt2_version().decode().startswith("libtt2_cpu")


@pytest.mark.parametrize("name,constraint", [("tacotron_small_freerun.npz", False),
                                             ("tacotron_small_window.npz", True)])
def test_golden_free_run(cpu, name, constraint):
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    g = _gold(name)
    B, T = g["ids"].shape
    n = int(g["max_iters"])
    eng = _taco(cpu, hp, W, B, T, g["ref_emt"].shape[1], n, constraint)
    out = eng.synthesize(g["ids"], g["lengths"], g["ref_emt"], g["ref_spk"], n, g["prenet_masks"])
    eng.close()
    np.testing.assert_allclose(out["mel_outputs"], g["mel_outputs"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(out["alignments"], g["alignments"], rtol=0, atol=1e-6)
    if "style" in g.files:
        np.testing.assert_allclose(out["style"], g["style"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(out["encoder_outputs"], g["encoder_outputs"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(out["stop_token_prediction"], g["stop_token_prediction"],
                                   rtol=0, atol=1e-6)


def test_golden_gta(cpu):
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    g = _gold("tacotron_small_gta.npz")
    B, T = g["ids"].shape
    n = int(g["max_iters"])
    eng = _taco(cpu, hp, W, B, T, g["ref_emt"].shape[1], n)
    out = eng.synthesize(g["ids"], g["lengths"], g["ref_emt"], g["ref_spk"], n, g["prenet_masks"],
                         0, g["targets"])
    eng.close()
    assert out["mel_outputs"].shape[1] == g["targets"].shape[1]
    for k in ("mel_outputs", "stop_token_prediction", "alignments"):
        np.testing.assert_allclose(out[k], g[k], rtol=0, atol=1e-5, err_msg=k)


def test_golden_decoder_step(cpu):
    hp = full_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    g = _gold("tacotron_decoder_step.npz")
    ids, lens = g["ids"], g["lengths"]
    eng = _taco(cpu, hp, W, ids.shape[0], ids.shape[1], g["ref_emt"].shape[1], 4)
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


def test_full_widths_monotonic_and_stop(cpu):
    """Fork widths, monotonic constraint (attention.py:205-207) and a stop bias near the boundary:
    the stop step and every output agree with the oracle."""
    hp = full_hparams()
    hp.synthesis_constraint_type = "monotonic"
    W = dict(init_tacotron_weights(hp, seed=5339))
    key = ("Tacotron_model/inference/decoder/stop_token_projection/"
           "projection_stop_token_projection/bias")
    W[key] = np.array([1.0], np.float32)
    B, T, n = 2, 9, 24
    ids, lens, re, rs = tacotron_inputs(B, T, 80, seed=5)
    masks = prenet_masks(n, B, 256, seed=5)
    eng = _taco(cpu, hp, W, B, T, 80, n, True)
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp, True), masks, n)
    assert out["mel_outputs"].shape == ref["mel_outputs"].shape
    for k in ("mel_outputs", "stop_token_prediction", "alignments"):
        np.testing.assert_allclose(out[k], ref[k], rtol=0, atol=1e-4, err_msg=k)


def test_seeded_masks_are_the_device_stream(cpu):
    """NULL prenet masks draw the rng.h stream keyed by seed — the bits tt2_prenet_keep_bits
    returns, shared with the HIP library by construction (one header)."""
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    B, T, n = 2, 7, 10
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=9)
    bits = np.zeros((n, 2, B, hp.prenet_layers[0]), np.uint8)
    _lib.check(cpu.tt2_prenet_keep_bits(77, n, B, hp.prenet_layers[0], _lib.ptr(bits)), cpu)
    assert 0.45 < bits.mean() < 0.55
    eng = _taco(cpu, hp, W, B, T, 64, n)
    a = eng.synthesize(ids, lens, re, rs, n, None, 77)
    b = eng.synthesize(ids, lens, re, rs, n, bits)
    eng.close()
    np.testing.assert_array_equal(a["mel_outputs"], b["mel_outputs"])


def test_errors_follow_the_abi(cpu):
    from tt2.engine import TacotronEngine
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    eng = TacotronEngine(hp, W, 2, 7, 64, 4, lib=cpu)
    with pytest.raises(_lib.TT2Error, match="before tt2_encode"):
        eng._B, eng._T_in = 2, 7
        eng.decode(4, prenet_masks(4, 2, hp.prenet_layers[0], seed=1))
    eng.close()
    W2 = dict(W)
    W2.pop("Tacotron_model/inference/memory_layer/kernel")
    with pytest.raises(_lib.TT2Error, match="memory_layer"):
        TacotronEngine(hp, W2, 2, 7, 64, 4, lib=cpu)


# ---------------------------------------------------------------- WaveNet
def test_golden_wavenet(cpu):
    from tt2.engine import WaveNetEngine
    hp = small_wavenet_hparams(6, 2)
    W = init_wavenet_weights(hp, seed=5339)
    g = _gold("wavenet_small_teacher.npz")
    B, T = g["teacher"].shape
    eng = WaveNetEngine(hp, W, B, T, lib=cpu)
    out = eng.generate(g["cond"], g["u_mix"], g["u_log"], 0, g["teacher"], want_logits=True,
                       want_upsampled=True)
    np.testing.assert_allclose(out["upsampled"], g["upsampled"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(out["logits"], g["logits"], rtol=0, atol=1e-5)
    np.testing.assert_array_equal(out["k"], g["k"])
    np.testing.assert_allclose(out["y"], g["y"], rtol=0, atol=1e-6)
    g2 = _gold("wavenet_small_freerun.npz")
    out2 = eng.generate(g2["cond"], g2["u_mix"], g2["u_log"], 0, None)
    eng.close()
    np.testing.assert_array_equal(out2["k"], g2["k"])
    np.testing.assert_allclose(out2["y"], g2["y"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("ut", ["1D", "Resize", "SubPixel", "NearestNeighbor"])
def test_wavenet_upsample_types(cpu, ut):
    from tt2.engine import WaveNetEngine
    hp = small_wavenet_hparams(4, 2)
    over = dict(upsample_type=ut)
    if ut == "SubPixel":
        over.update(NN_init=False, upsample_activation="LeakyRelu")
    hp.override_from_dict(over)
    W = init_wavenet_weights(hp, seed=5339)
    B, T_f = 2, 2
    hop = int(np.prod(hp.upsample_scales))
    T = T_f * hop
    rng = np.random.default_rng(4)
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32))
    um, ul = mol_uniforms(T, B, seed=4)
    eng = WaveNetEngine(hp, W, B, T, lib=cpu)
    out = eng.generate(cond, um, ul, 0, None, want_logits=True, want_upsampled=True)
    eng.close()
    oh = wavenet_oracle_hp(hp)
    c_up = WR.upsample_network(cond.transpose(0, 2, 1), W, oh)
    np.testing.assert_allclose(out["upsampled"], c_up, rtol=0, atol=1e-5)
    y, k, lg = WR.incremental(c_up.transpose(0, 2, 1), W, oh, um, ul, return_logits=True)
    np.testing.assert_allclose(out["logits"], lg, rtol=0, atol=1e-4)
    np.testing.assert_array_equal(out["k"], k)


def test_golden_mol_sampler(cpu):
    g = _gold("mol_sampler.npz")
    n = g["logits"].shape[0]
    x = np.zeros(n, np.float32)
    k = np.zeros(n, np.int32)
    _lib.check(cpu.tt2_mol_sample(_lib.ptr(np.ascontiguousarray(g["logits"])),
                                  _lib.ptr(np.ascontiguousarray(g["u_mix"])),
                                  _lib.ptr(np.ascontiguousarray(g["u_log"])), n, 10,
                                  float(g["log_scale_min"]), _lib.ptr(x), _lib.ptr(k)), cpu)
    np.testing.assert_array_equal(k, g["k"])                   # the mixture choice: exact
    np.testing.assert_allclose(x, g["x"], rtol=0, atol=1e-6)   # expf / fused multiply-add rounding


@pytest.mark.parametrize("style", ["embed", "adain"])
def test_style_paths(cpu, style):
    """The non-GST style paths (tacotron.py:236-308) at both widths, emotion and speaker
    references of different lengths: 'embed' (args.pretrained_emb_disc_all / use_gst=False) and
    'adain' (ReferenceEncoderAdaIn, modules.py:66-107)."""
    from tt2.engine import TacotronEngine
    for hp in (small_hparams(), full_hparams()):
        W = init_tacotron_weights(hp, seed=5339, style=style)
        B, T, n = 3, 11, 8
        ids, lens, re, rs = tacotron_inputs(B, T, 100, seed=12)
        rs = np.ascontiguousarray(rs[:, :72])
        masks = prenet_masks(n, B, hp.prenet_layers[0], seed=12)
        eng = TacotronEngine(hp, W, B, T, 100, n, lib=cpu, style=style)
        out = eng.synthesize(ids, lens, re, rs, n, masks)
        eng.close()
        ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp, style=style), masks, n)
        np.testing.assert_allclose(out["style"], ref["style"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], rtol=0, atol=1e-4)


def test_use_gst_false_is_embed(cpu):
    """hp.use_gst=False selects the reference embeddings (tacotron.py:269, 284-291)."""
    from tt2.engine import TacotronEngine
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339, style="embed")
    hp.use_gst = False
    B, T, n = 2, 7, 5
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=13)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=13)
    eng = TacotronEngine(hp, W, B, T, 64, n, lib=cpu)
    assert eng.D == 2 * hp.encoder_lstm_units + 256
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("constraint", [False, True])
def test_smoothing_normalization_matches_oracle(cpu, constraint):
    """hp.smoothing: _smoothing_normalization (attention.py:71-80, chosen at :150) = sigmoid(e) /
    sum_j sigmoid(e) instead of softmax; masked scores (length mask -inf, window -2^32+1) get 0."""
    hp = small_hparams()
    hp.override_from_dict(dict(smoothing=True))
    W = init_tacotron_weights(hp, seed=5339)
    B, T, n = 3, 11, 9
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=71)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=71)
    eng = _taco(cpu, hp, W, B, T, 40, n, constraint)
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp, constraint), masks, n)
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], rtol=0, atol=1e-5)
    al = ref["alignments"]                      # [B, T_in, n]
    np.testing.assert_allclose(al.sum(axis=1), 1.0, atol=1e-5)
    for b in range(B):
        assert np.all(al[b, lens[b]:] == 0)
    # a different normalisation than softmax: the same weights without smoothing differ
    hp.override_from_dict(dict(smoothing=False))
    ref0 = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp, constraint), masks, n)
    assert np.abs(ref0["alignments"] - al).max() > 1e-3


def test_chunk_ranges_and_global_stop():
    """Row chunks of a tower above one context's 32 rows, and the tower-level stop step
    (TacoTestHelper, helpers.py:40-54: every row's rounded stop token; stop_at_any reduces over the r
    frames of a step AFTER the batch axis, so at r = 1 it changes nothing)."""
    from tt2.engine import chunk_ranges, global_stop_steps
    assert chunk_ranges(32) == [(0, 32)]
    assert chunk_ranges(33) == [(0, 17), (17, 33)]
    assert chunk_ranges(96) == [(0, 32), (32, 64), (64, 96)]
    assert chunk_ranges(65) == [(0, 22), (22, 44), (44, 65)]
    st = np.full((4, 9), 0.2, np.float32)
    assert global_stop_steps(st, False) == 9 and global_stop_steps(st, True) == 9
    st[1, 3] = 0.9                       # one row only: no stop, with or without stop_at_any
    assert global_stop_steps(st, True) == 9 and global_stop_steps(st, False) == 9
    st[:, 6] = 0.75
    assert global_stop_steps(st, False) == 7 and global_stop_steps(st, True) == 7
    st[:, 5] = 0.5                       # tf.round: half to even -> 0, no stop at step 5
    assert global_stop_steps(st, False) == 7


@pytest.mark.parametrize("stop_at_any,bias,scale,steps", [(False, -6.0, 1, 12), (True, -3.0, 30, 12),
                                                         (False, 4.0, 1, 1), (True, 4.0, 1, 1)])
def test_chunked_tower_matches_oracle(cpu, stop_at_any, bias, scale, steps):
    """A 40-row tower (two 20-row contexts, no stop rule of their own) against one oracle decode
    of all 40 rows: frames, alignments and the tower's stop step.  The stop
    projection is biased / scaled so the rule never fires, fires mid-run on a few rows only (no stop:
    every row must round to 1, stop_at_any or not -- helpers.py:40-54 at r = 1), or fires on every
    row at the first step."""
    from tt2.engine import TacotronEngine
    from _common import STOP_BIAS
    hp = small_hparams()
    hp.override_from_dict(dict(stop_at_any=stop_at_any))
    W = init_tacotron_weights(hp, seed=5339)
    W[STOP_BIAS] = np.full((1,), bias, np.float32)
    K = STOP_BIAS.replace("/bias", "/kernel")
    W[K] = W[K] * scale
    B, T, n = 40, 9, 12
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=17)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=17)
    eng = TacotronEngine(hp, W, B, T, 40, n, lib=cpu)
    assert eng._chunks is not None and [c.caps[0] for c in eng._chunks] == [20, 20]
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    assert ref["mel_outputs"].shape[1] == steps
    assert out["mel_outputs"].shape == ref["mel_outputs"].shape
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(out["stop_token_prediction"], ref["stop_token_prediction"], rtol=0,
                               atol=1e-5)
