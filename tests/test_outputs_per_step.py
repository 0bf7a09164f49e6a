"""outputs_per_step r > 1 (hparams.py:140): FrameProjection(num_mels * r) / StopProjection(shape=r)
(tacotron.py:322-324), the step's last frame fed back (helpers.py:57), every r-th target frame under
GTA (helpers.py:78) and the [B, r] stop rule (helpers.py:40-54), on the oracle, the host backend and
the HIP launch path (VERDICT r05 "what's missing" 1)."""
import os
import subprocess

import numpy as np
import pytest

from _common import oracle_hp, prenet_masks, small_hparams, full_hparams, tacotron_inputs
from oracle import tacotron_ref as TR
from tt2 import _lib
from tt2.weights import init_tacotron_weights

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PFX = "Tacotron_model/inference/decoder/"
FK = PFX + "linear_transform_projection/projection_linear_transform_projection/kernel"
FB = PFX + "linear_transform_projection/projection_linear_transform_projection/bias"
SK = PFX + "stop_token_projection/projection_stop_token_projection/kernel"
SB = PFX + "stop_token_projection/projection_stop_token_projection/bias"


def _hp(r, full=False, **kw):
    hp = full_hparams() if full else small_hparams()
    hp.override_from_dict(dict(outputs_per_step=r, **kw))
    return hp


def _weights(hp, seed=5339, stop_bias=None):
    W = dict(init_tacotron_weights(hp, seed=seed))
    if stop_bias is not None:
        W[SB] = np.asarray(stop_bias, np.float32).reshape(hp.outputs_per_step)
    return W


def _duplicated(W1, r):
    """r-frame weights whose r frame / stop column groups all repeat the r = 1 model's: the r = r
    decode then emits each r = 1 frame r times and feeds the same frame back."""
    W = dict(W1)
    W[FK] = np.tile(W1[FK], (1, r))
    W[FB] = np.tile(W1[FB], r)
    W[SK] = np.tile(W1[SK], (1, r))
    W[SB] = np.tile(W1[SB], r)
    return W


# ---------------------------------------------------------------- oracle
@pytest.mark.parametrize("r", [2, 3])
def test_oracle_duplicated_columns_reduce_to_r1(r):
    """Property pinning the oracle's r handling against its r = 1 path: with every frame / stop
    column group equal, frames[:, i::r] are the r = 1 frames, the stop step is the same and GTA on
    targets T feeds targets[:, r-1::r] exactly as r = 1 GTA on those frames."""
    hp1 = small_hparams()
    W1 = _weights(hp1)
    W = _duplicated(W1, r)
    B, T, n = 3, 9, 8
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=3)
    masks = prenet_masks(n, B, hp1.prenet_layers[0], seed=3)
    o1 = TR.synthesize(ids, lens, re, rs, W1, oracle_hp(hp1), masks, n)
    orr = TR.synthesize(ids, lens, re, rs, W, oracle_hp(_hp(r)), masks, n)
    n1 = o1["alignments"].shape[2]
    assert orr["alignments"].shape[2] == n1
    assert orr["decoder_output"].shape == (B, n1 * r, hp1.num_mels)
    for i in range(r):
        np.testing.assert_allclose(orr["decoder_output"][:, i::r], o1["decoder_output"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(orr["stop_token_prediction"][:, i::r], o1["stop_token_prediction"],
                                   rtol=0, atol=1e-6)
    np.testing.assert_allclose(orr["alignments"], o1["alignments"], rtol=0, atol=1e-6)
    rng = np.random.default_rng(4)
    tg = rng.uniform(-4, 4, (B, n * r + 1, hp1.num_mels)).astype(np.float32)   # ragged tail dropped
    g1 = TR.synthesize(ids, lens, re, rs, W1, oracle_hp(hp1), masks, n, targets=tg[:, r - 1::r][:, :n])
    gr = TR.synthesize(ids, lens, re, rs, W, oracle_hp(_hp(r)), masks, n, targets=tg)
    assert gr["decoder_output"].shape[1] == n * r
    np.testing.assert_allclose(gr["decoder_output"][:, r - 1::r], g1["decoder_output"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("stop_at_any", [False, True])
def test_oracle_stop_rule_any_all_over_r_frames(stop_at_any):
    """helpers.py:51-54: stop_at_any = reduce_any over the r frames of reduce_all over the batch;
    otherwise reduce_all.  Frame 0's stop token always rounds to 1, frame 1's never: stop_at_any
    stops after the first step, the safe rule runs to max_iters."""
    hp = _hp(2, stop_at_any=stop_at_any)
    W = _weights(hp, stop_bias=[40.0, -40.0])
    B, T, n = 2, 7, 6
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=5)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=5)
    o = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    assert o["alignments"].shape[2] == (1 if stop_at_any else n)


# ---------------------------------------------------------------- host backend (libtt2_cpu.so)
@pytest.fixture(scope="module")
def cpu():
    if not os.path.exists(_lib.CPU_LIB_PATH):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "tacotron-2_amd"), "libtt2_cpu.so"])
    return _lib.load_cpu_library()


def _run(hp, W, B, T, n, seed, lib=None, targets=None, stop_at_any=None):
    from tt2.engine import TacotronEngine
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=seed)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=seed)
    eng = TacotronEngine(hp, W, B, T, 40, n, lib=lib)
    try:
        out = eng.synthesize(ids, lens, re, rs, n, masks, 0, targets)
        path = eng.decoder_path()[0] if lib is None else None
    finally:
        eng.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n, targets=targets)
    return out, ref, path


def _check(out, ref, atol_mel=1e-4, atol_align=1e-5):
    assert out["mel_outputs"].shape == ref["mel_outputs"].shape
    np.testing.assert_allclose(out["decoder_output"], ref["decoder_output"], rtol=0, atol=atol_mel)
    np.testing.assert_allclose(out["mel_outputs"], ref["mel_outputs"], rtol=0, atol=atol_mel)
    np.testing.assert_allclose(out["stop_token_prediction"], ref["stop_token_prediction"], rtol=0,
                               atol=atol_align)
    np.testing.assert_allclose(out["alignments"], ref["alignments"], rtol=0, atol=atol_align)


@pytest.mark.parametrize("r,stop_at_any,bias", [(2, False, 0.0), (2, True, 0.5), (3, False, -6.0),
                                                (2, True, [40.0, -40.0]), (2, False, [40.0, -40.0])])
def test_cpu_backend_matches_oracle(cpu, r, stop_at_any, bias):
    hp = _hp(r, stop_at_any=stop_at_any)
    W = _weights(hp, stop_bias=np.broadcast_to(np.float32(bias), (r,)) if np.ndim(bias) == 0 else bias)
    out, ref, _ = _run(hp, W, 3, 9, 10, 21, cpu)
    _check(out, ref)


@pytest.mark.parametrize("r,T_tg", [(2, 14), (3, 17)])
def test_cpu_backend_gta_matches_oracle(cpu, r, T_tg):
    hp = _hp(r)
    W = _weights(hp)
    tg = np.random.default_rng(8).uniform(-4, 4, (3, T_tg, hp.num_mels)).astype(np.float32)
    out, ref, _ = _run(hp, W, 3, 9, 12, 23, cpu, targets=tg)
    assert out["mel_outputs"].shape[1] == (T_tg // r) * r
    _check(out, ref)


def test_cpu_backend_chunked_tower_r2(cpu):
    """A 40-row tower (two contexts without their own stop rule) at r = 2: the host takes the
    tower's stop step over all rows' [B, r] stop tokens."""
    hp = _hp(2, stop_at_any=True)
    W = _weights(hp, stop_bias=[-3.0, -3.0])
    W[SK] = W[SK] * 30
    out, ref, _ = _run(hp, W, 40, 9, 12, 17, cpu)
    _check(out, ref)


def test_global_stop_steps_over_r_frames():
    from tt2.engine import global_stop_steps
    st = np.full((3, 5 * 2), 0.2, np.float32)            # [B, n * r], r = 2
    assert global_stop_steps(st, False, 2) == 5 and global_stop_steps(st, True, 2) == 5
    st[:, 4] = 0.9                                        # frame 0 of step 2 on every row
    assert global_stop_steps(st, True, 2) == 3 and global_stop_steps(st, False, 2) == 5
    st[:, 5] = 0.9                                        # both frames of step 2
    assert global_stop_steps(st, False, 2) == 3
    st[1, 5] = 0.5                                        # half to even: one row not finished
    assert global_stop_steps(st, False, 2) == 5 and global_stop_steps(st, True, 2) == 3


def test_config_carries_r_and_rejects_out_of_range(cpu):
    from tt2.engine import TacotronEngine, tacotron_config
    hp = _hp(3)
    assert tacotron_config(hp, 2, 9, 40, 5, lib=cpu).outputs_per_step == 3
    hp9 = _hp(9)
    with pytest.raises(_lib.TT2Error, match="outputs_per_step"):
        TacotronEngine(hp9, _weights(hp9), 2, 9, 40, 5, lib=cpu)


# ---------------------------------------------------------------- HIP launch path
@pytest.mark.gpu
@pytest.mark.parametrize("r,stop_at_any,bias,full", [(2, False, 0.0, False), (3, True, 0.5, False),
                                                     (2, True, [40.0, -40.0], False),
                                                     (2, False, -6.0, True), (3, False, 0.3, True)])
def test_gpu_launch_path_matches_oracle(r, stop_at_any, bias, full):
    """r > 1 decodes on the per-step launch path (tacotron.hip k_proj: nm·r frame columns, the r
    stop columns in one tile, W1 folded through the last frame's columns) at the small and the fork
    widths; outputs within the launch path's r = 1 tolerances of the float32 oracle."""
    hp = _hp(r, full, stop_at_any=stop_at_any)
    W = _weights(hp, stop_bias=np.broadcast_to(np.float32(bias), (r,)) if np.ndim(bias) == 0 else bias)
    out, ref, path = _run(hp, W, 3, 11, 14, 31)
    assert path == 0
    _check(out, ref, 2e-4 if full else 1e-4, 2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("r,T_tg,full", [(2, 22, False), (3, 25, True)])
def test_gpu_gta_matches_oracle(r, T_tg, full):
    hp = _hp(r, full)
    W = _weights(hp)
    tg = np.random.default_rng(9).uniform(-4, 4, (3, T_tg, hp.num_mels)).astype(np.float32)
    out, ref, path = _run(hp, W, 3, 11, 12, 33, targets=tg)
    assert path == 0 and out["mel_outputs"].shape[1] == min(12, T_tg // r) * r
    _check(out, ref, 2e-4 if full else 1e-4, 2e-5)


@pytest.mark.gpu
def test_gpu_chunked_tower_r2_matches_oracle():
    hp = _hp(2, stop_at_any=True)
    W = _weights(hp, stop_bias=[-3.0, -3.0])
    W[SK] = W[SK] * 30
    out, ref, _ = _run(hp, W, 40, 9, 12, 17)
    _check(out, ref)


@pytest.mark.gpu
def test_gpu_duplicated_columns_reduce_to_r1():
    """The same reduction property on the device: the r = 2 launch path with duplicated column
    groups reproduces the r = 1 decode of the same model frame for frame (the persistent decoder
    serves r = 1 at these widths; the launch path serves r = 2)."""
    from tt2.engine import TacotronEngine
    hp1 = full_hparams()
    W1 = _weights(hp1)
    W2 = _duplicated(W1, 2)
    B, T, n = 4, 13, 16
    ids, lens, re, rs = tacotron_inputs(B, T, 40, seed=41)
    masks = prenet_masks(n, B, 256, seed=41)
    outs = []
    for hp, W in ((hp1, W1), (_hp(2, True), W2)):
        eng = TacotronEngine(hp, W, B, T, 40, n)
        outs.append(eng.synthesize(ids, lens, re, rs, n, masks))
        eng.close()
    o1, o2 = outs
    assert o2["decoder_output"].shape[1] == 2 * o1["decoder_output"].shape[1]
    for i in range(2):
        np.testing.assert_allclose(o2["decoder_output"][:, i::2], o1["decoder_output"], rtol=0, atol=2e-4)
