"""outputs_per_step r > 1 in the training step (hparams.py:140): FrameProjection(num_mels * r) and
StopProjection(shape=r) per decoder step (tacotron.py:322-324), decoder_output / stop reshaped to
[B, T·r, ..] (tacotron.py:355-358), TacoTrainingHelper feeding targets[:, r-1::r] (helpers.py:78)
or the last of the step's own r frames (helpers.py:129), the loss masks rounded up to a multiple of
r (modules.py:523-530).

CPU: the float64 restatement (oracle/train_ref.py) against the numpy inference oracle's GTA decode
at r > 1, against its own r = 1 path on duplicated projection columns, and its gradients against
central differences.  GPU: libtt2's training step (csrc/train.hip) at r = 2 / 3 against that
oracle -- small widths in fp32 with free-running steps, ragged masked lengths and the Postnet, and
the fork widths in bf16 through the persistent forward / backward.  Parity unpinned against TF
itself."""
import numpy as np
import pytest
import torch

from _common import small_hparams
from oracle import tacotron_ref as TR
from oracle import train_ref as TRN
from oracle.hp import oracle_hp
from test_train import _clip, _rel
from tt2.synthetic import postnet_masks, prenet_masks, train_batch, zoneout_masks
from tt2.train import draw_teacher_forcing, train_config
from tt2.weights import init_tacotron_weights, memory_width

MEM_K = "Tacotron_model/inference/memory_layer/kernel"


def _hp(r, full=False, **kw):
    if full:
        from tt2.hparams import hparams
        hp = hparams.copy()
        hp.override_from_dict(dict(tacotron_num_gpus=1))
    else:
        hp = small_hparams()
    hp.override_from_dict(dict(outputs_per_step=r, **kw))
    return hp


def _case(hp, B, T_in, T_out, seed=11):
    """T_out frames; the prenet / zoneout masks are per decoder step (T_out / r)."""
    r = hp.outputs_per_step
    assert T_out % r == 0
    W = init_tacotron_weights(hp, seed=5339)
    mem, lens, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=seed)
    pm = prenet_masks(T_out // r, B, hp.prenet_layers[0], seed=seed)
    zm = zoneout_masks(T_out // r, B, hp.decoder_lstm_units, seed=seed)
    return W, mem, lens, tg, st, pm, zm


def _t64(x):
    return torch.tensor(np.asarray(x), dtype=torch.float64)


# ---------------------------------------------------------------- oracle (CPU)
@pytest.mark.parametrize("r", [2, 3])
def test_oracle_train_forward_r_is_the_gta_decode(r):
    """With inference zoneout the restatement at r is the numpy oracle's GTA decode at r
    (dynamic_decode with targets: every r-th target frame fed, r frames / stops per step)."""
    hp = _hp(r)
    T_out = 4 * r
    W, mem, lens, tg, st, pm, _ = _case(hp, 3, 9, T_out)
    Wt = {n: _t64(W[n]) for n in TRN.train_var_names()}
    fr, sl, al = TRN.forward(Wt, _t64(mem), lens, _t64(tg), _t64(pm), None, zoneout=hp.tacotron_zoneout_rate)
    assert fr.shape == (3, T_out, hp.num_mels) and sl.shape == (3, T_out) and al.shape == (3, 9, 4)
    mask = (np.arange(mem.shape[1])[None, :] < lens[:, None])
    values = mem.astype(np.float64) * mask[:, :, None]
    keys = values @ np.asarray(W[MEM_K], np.float64)
    f2, s2, a2 = TR.dynamic_decode(keys, values, lens, W, oracle_hp(hp), pm, T_out // r, targets=tg,
                                   dt=np.float64)
    np.testing.assert_allclose(fr.numpy(), f2, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(torch.sigmoid(sl).numpy(), s2, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(al.numpy(), a2, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("r", [2, 3])
def test_oracle_train_duplicated_columns_reduce_to_r1(r):
    """Property pinning the r handling against the r = 1 restatement: with every frame / stop
    column group equal to the r = 1 model's, frames[:, i::r] are the r = 1 frames on the targets
    targets[:, r-1::r], including free-running steps (the fed-back frame is the last of the r)."""
    hp1 = small_hparams()
    n = 4
    W1, mem, lens, tg, st, pm, zm = _case(hp1, 2, 7, n * r)
    FP, SP = TRN.FP, TRN.SP
    Wr = dict(W1)
    Wr[FP + "kernel"] = np.tile(W1[FP + "kernel"], (1, r))
    Wr[FP + "bias"] = np.tile(W1[FP + "bias"], r)
    Wr[SP + "kernel"] = np.tile(W1[SP + "kernel"], (1, r))
    Wr[SP + "bias"] = np.tile(W1[SP + "bias"], r)
    pm, zm = pm[:n], zm[:n]
    feed = np.array([1, 0, 1, 0], np.uint8)
    W1t = {k: _t64(W1[k]) for k in TRN.train_var_names()}
    Wrt = {k: _t64(Wr[k]) for k in TRN.train_var_names()}
    f1, s1, a1 = TRN.forward(W1t, _t64(mem), lens, _t64(tg[:, r - 1::r]), _t64(pm), _t64(zm), feed_target=feed)
    fr, sr, ar = TRN.forward(Wrt, _t64(mem), lens, _t64(tg), _t64(pm), _t64(zm), feed_target=feed)
    for i in range(r):  # (the wider products may sum in another order: float64 rounding only)
        torch.testing.assert_close(fr[:, i::r], f1, rtol=0, atol=1e-12)
        torch.testing.assert_close(sr[:, i::r], s1, rtol=0, atol=1e-12)
    torch.testing.assert_close(ar, a1, rtol=0, atol=1e-12)


def test_oracle_train_r_gradients_match_finite_differences():
    """r = 2 with free-running steps (gradient through the last of the fed-back r frames), masked
    losses over ragged lengths, pos_weight and the Postnet: autograd against central differences
    on the r-wide projections and the prenet."""
    hp = _hp(2)
    W, mem, lens, tg, st, pm, zm = _case(hp, 2, 6, 8)
    feed = np.array([1, 0, 1, 0], np.uint8)
    tl = np.array([7, 4])                                              # max 7 -> rounded up to 8
    pnm = postnet_masks(hp.postnet_num_layers, 2, 8, hp.postnet_channels, seed=1)
    _, _, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, reg_weight=1e-3, postnet=True, postnet_masks=pnm,
                              feed_target=feed, target_lengths=tl, pos_weight=7.0)

    def loss_of(W2):
        names = TRN.train_var_names() + TRN.postnet_var_names()
        Wt = {k: _t64(W2[k]) for k in names}
        fr, sl, _ = TRN.forward(Wt, _t64(mem), lens, _t64(tg), _t64(pm), _t64(zm), feed_target=feed)
        b, s, r = TRN.losses(fr, sl, _t64(tg), _t64(st), Wt, 1e-3, target_lengths=tl, pos_weight=7.0)
        dec = TRN.clip_decoder_output(fr)
        proj, _ = TRN.postnet_train(Wt, dec, _t64(pnm))
        after = TRN.masked_mse(_t64(tg), TRN.clip_decoder_output(dec + proj), tl)
        return float(b + s + r + after)

    rng = np.random.default_rng(5)
    nm = hp.num_mels
    for name, cols in [(TRN.FP + "kernel", (0, 2 * nm)), (TRN.FP + "kernel", (nm, 2 * nm)),
                       (TRN.FP + "bias", (nm, 2 * nm)), (TRN.SP + "kernel", (0, 2)), (TRN.SP + "bias", (0, 2)),
                       (TRN.P + "decoder/decoder_prenet/dense_1/kernel", None)]:
        arr = np.asarray(W[name], np.float64)
        for _ in range(2):
            idx = tuple(int(rng.integers(0, s)) for s in arr.shape)
            if cols is not None:
                idx = idx[:-1] + (int(rng.integers(*cols)),)
            eps = 1e-6
            Wp, Wm = dict(W), dict(W)
            ap, am = arr.copy(), arr.copy()
            ap[idx] += eps
            am[idx] -= eps
            Wp[name], Wm[name] = ap, am
            fd = (loss_of(Wp) - loss_of(Wm)) / (2 * eps)
            assert abs(fd - g[name][idx]) < 1e-6 + 1e-4 * abs(fd), (name, idx, fd, g[name][idx])


def test_train_config_outputs_per_step():
    assert train_config(_hp(3), 2, 8, 9).outputs_per_step == 3
    assert train_config(small_hparams(), 2, 8, 9).outputs_per_step == 1


# ---------------------------------------------------------------- libtt2 (GPU)
def _run(hp, W, case, T_in, T_out, postnet, feed=None, tl=None, pnm=None, precision="fp32"):
    from tt2.train import TacotronTrainer
    mem, lens, tg, st, pm, zm = case
    B = tg.shape[0]
    names = TRN.train_var_names() + (TRN.postnet_var_names() if postnet else [])
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, postnet=postnet, precision=precision)
    try:
        tr.set_step_inputs(targets_lengths=tl, feed_target=feed)
        tr.forward_backward(mem, lens, tg, st, pm, zm, pnm)
        L = tr.losses()
        fr, sl, al = tr.outputs(T_in, T_out)
        mel = tr.mel_outputs(T_out) if postnet else None
        grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
        gmem = tr.get("memory", 1, mem.shape)
        persist = (float(tr.get("diag:persist", 0, (1,))[0]), float(tr.get("diag:persist_bwd", 0, (1,))[0]))
    finally:
        tr.close()
    return dict(L=L, fr=fr, sl=sl, al=al, mel=mel, g=grads, gmem=gmem, names=names, persist=persist)


@pytest.mark.gpu
@pytest.mark.parametrize("r,postnet", [(2, True), (2, False), (3, True)])
def test_gpu_train_outputs_per_step_matches_oracle(r, postnet):
    """fp32 step at r frames per decoder step, small widths: free-running steps (the last of the
    step's r frames fed back), ragged masked lengths whose maximum rounds up to T_out, pos_weight
    20 and (postnet) the Postnet over all T·r frames -- frames / stop logits / alignments within
    1e-4, losses within 1e-5 relative, every gradient (incl. d memory) within 2e-4 of the float64
    oracle (the tolerances of test_gpu_train_teacher_forcing_and_masked_losses)."""
    hp = _hp(r, mask_decoder=True, cross_entropy_pos_weight=20.0)
    B, T_in, T_out = 3, 9, 4 * r
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out, seed=29)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=29) if postnet else None
    feed = draw_teacher_forcing(T_out // r, 0.5, np.random.default_rng(4))
    feed[1], feed[2] = 0, 1                                            # both kinds present
    tl = np.array([T_out - 1, 5, 2], np.int32)
    res = _run(hp, W, (mem, lens, tg, st, pm, zm), T_in, T_out, postnet, feed, tl, pnm)
    out, Lr, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp),
                                 postnet=postnet, postnet_masks=pnm, feed_target=feed, target_lengths=tl,
                                 pos_weight=20.0)
    assert res["fr"].shape == (B, T_out, hp.num_mels) and res["al"].shape == (B, T_in, T_out // r)
    assert np.abs(res["fr"] - out["frames"]).max() < 1e-4
    assert np.abs(res["sl"] - out["stop_logits"]).max() < 1e-4
    assert np.abs(res["al"] - out["alignments"]).max() < 1e-4
    L = res["L"]
    assert abs(L["before"] - Lr[0]) < 1e-5 * Lr[0] and abs(L["stop_token"] - Lr[1]) < 1e-5 * Lr[1]
    if postnet:
        assert abs(L["after"] - Lr[3]) < 1e-5 * Lr[3]
        assert np.abs(res["mel"] - out["mel_outputs"]).max() < 1e-4
    for n in res["names"]:
        if np.abs(g[n]).max() < 1e-12:
            assert np.abs(res["g"][n]).max() < 1e-6, n
            continue
        assert _rel(res["g"][n], g[n]) < 2e-4, (n, _rel(res["g"][n], g[n]))
    assert _rel(res["gmem"], g["memory"]) < 2e-4


@pytest.mark.gpu
def test_gpu_train_outputs_per_step_shape_errors():
    """T_out must be a multiple of r (the feeder pads to one) and, under mask_decoder, the longest
    target length rounded up to r must equal T_out (sequence_mask, modules.py:523-530)."""
    from tt2._lib import TT2Error
    from tt2.train import TacotronTrainer
    hp = _hp(2, mask_decoder=True)
    W, mem, lens, tg, st, pm, zm = _case(hp, 2, 6, 8)
    tr = TacotronTrainer(hp, W, 2, 6, 8, 0, postnet=False)
    try:
        with pytest.raises(ValueError, match="multiple of outputs_per_step"):
            tr.forward_backward(mem, lens, tg[:, :7], st[:, :7], pm, zm)
        with pytest.raises(ValueError, match="prenet_masks"):
            tr.forward_backward(mem, lens, tg, st, np.concatenate([pm, pm]), zm)
        tr.set_step_inputs(targets_lengths=np.array([6, 3]))           # rounds up to 6 != 8
        with pytest.raises(TT2Error, match="rounded up"):
            tr.forward_backward(mem, lens, tg, st, pm, zm)
        tr.set_step_inputs(targets_lengths=np.array([7, 3]))           # rounds up to 8
        tr.forward_backward(mem, lens, tg, st, pm, zm)
        assert np.isfinite(tr.losses()["loss"])
    finally:
        tr.close()


@pytest.mark.gpu
def test_gpu_train_outputs_per_step_fork_widths_bf16_persistent():
    """r = 2 at the fork widths in the bf16 step: the persistent forward and backward (r-agnostic:
    they see decoder steps) with the r-wide projections, losses and Postnet around them, against
    the float64 oracle at the mixed-precision tolerances of
    test_gpu_train_persistent_forward_close_to_oracle."""
    hp = _hp(2, full=True)
    B, T_in, T_out = 8, 37, 32
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    res = _run(hp, W, (mem, lens, tg, st, pm, zm), T_in, T_out, False, precision="bf16")
    assert res["persist"] == (1.0, 1.0)
    out, (b, s, _), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp))
    assert np.abs(res["al"] - out["alignments"]).max() < 1e-3
    assert np.abs(res["fr"] - out["frames"]).max() < 1e-2
    assert abs(res["L"]["before"] - b) < 1e-3 * b and abs(res["L"]["stop_token"] - s) < 1e-3 * s
    for n in TRN.train_var_names():
        frob = float(np.linalg.norm(res["g"][n] - g[n]) / max(np.linalg.norm(g[n]), 1e-30))
        print("  {:90s} frob {:.3e}".format(n, frob))
        assert frob < (0.1 if "prenet" in n else 1e-2), (n, frob)
