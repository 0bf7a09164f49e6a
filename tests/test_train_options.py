"""Training-step options beyond the default hparams (round 3): the teacher-forcing draw with
constant / scheduled ratio (TacoTrainingHelper, helpers.py:60-180; hparams.py:300-307) and the
masked losses with the stop-token pos_weight (mask_decoder / cross_entropy_pos_weight,
tacotron.py:56,758-767, modules.py:523-575; hparams.py:192-193).

CPU: the oracle's restatement of both (oracle/train_ref.py) against hand-computed values and
central finite differences, the product-side schedule and draw.  GPU: libtt2's training step
(csrc/train.hip) with free-running steps, ragged target lengths and pos_weight against the
float64 oracle.  Parity unpinned against TF itself."""
import numpy as np
import pytest
import torch

from _common import small_hparams
from oracle import train_ref as TRN
from test_train import _case, _clip, _rel
from tt2.synthetic import postnet_masks
from tt2.train import draw_teacher_forcing, teacher_forcing_ratio, train_config


def test_teacher_forcing_ratio_schedule():
    """'constant' = tacotron_teacher_forcing_ratio; 'scheduled' = init before start_decay, then
    init·rate^((step - start)/decay_steps) (tf.train.exponential_decay, not staircase) -- the
    product's schedule and the oracle's agree at every step."""
    hp = small_hparams()
    assert teacher_forcing_ratio(123456, hp) == 1.0                  # fork default: constant 1
    hp.override_from_dict(dict(tacotron_teacher_forcing_ratio=0.75))
    assert teacher_forcing_ratio(0, hp) == 0.75
    hp.override_from_dict(dict(tacotron_teacher_forcing_mode="scheduled"))
    for step, want in [(0, 1.0), (9999, 1.0), (10000, 1.0), (50000, 0.1), (30000, 0.1 ** 0.5)]:
        assert abs(teacher_forcing_ratio(step, hp) - want) < 1e-12, step
        assert abs(TRN.teacher_forcing_ratio(step, hp) - want) < 1e-12, step
    hp.override_from_dict(dict(tacotron_teacher_forcing_mode="cosine"))
    with pytest.raises(ValueError):
        teacher_forcing_ratio(0, hp)


def test_draw_teacher_forcing():
    rng = np.random.default_rng(0)
    assert draw_teacher_forcing(50, 1.0, rng).all()
    f0 = draw_teacher_forcing(50, 0.0, rng)
    assert f0[0] == 1 and not f0[1:].any()                          # go frame, then own frames
    f = draw_teacher_forcing(20000, 0.3, rng)
    assert f.dtype == np.uint8 and abs(f[1:].mean() - 0.3) < 0.02


def test_train_config_accepts_the_options():
    hp = small_hparams()
    hp.override_from_dict(dict(mask_decoder=True, cross_entropy_pos_weight=20,
                               tacotron_teacher_forcing_mode="scheduled"))
    cfg = train_config(hp, 2, 8, 8)
    assert cfg.mask_decoder == 1 and cfg.pos_weight == 20.0
    hp.override_from_dict(dict(predict_linear=True))
    with pytest.raises(NotImplementedError):
        train_config(hp, 2, 8, 8)


def _t64(x):
    return torch.tensor(np.asarray(x), dtype=torch.float64)


def test_oracle_all_teacher_forced_draw_is_the_default_forward():
    hp = small_hparams()
    W, mem, lens, tg, st, pm, zm = _case(hp, B=2, T_in=6, T_out=5)
    Wt = {n: _t64(W[n]) for n in TRN.train_var_names()}
    a = TRN.forward(Wt, _t64(mem), lens, _t64(tg), _t64(pm), _t64(zm))
    b = TRN.forward(Wt, _t64(mem), lens, _t64(tg), _t64(pm), _t64(zm), feed_target=np.ones(5, np.uint8))
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_oracle_free_running_step_feeds_the_unclipped_frame():
    """A step with feed 0 consumes the decoder's own previous frame: changing the target frame
    t-1 leaves every output up to and including step t unchanged when step t runs free."""
    hp = small_hparams()
    W, mem, lens, tg, st, pm, zm = _case(hp, B=2, T_in=6, T_out=5)
    Wt = {n: _t64(W[n]) for n in TRN.train_var_names()}
    feed = np.array([1, 1, 0, 1, 1], np.uint8)
    tg2 = tg.copy()
    tg2[:, 1] += 3.0                                                  # target frame 1 feeds step 2 only
    f1, _, _ = TRN.forward(Wt, _t64(mem), lens, _t64(tg), _t64(pm), _t64(zm), feed_target=feed)
    f2, _, _ = TRN.forward(Wt, _t64(mem), lens, _t64(tg2), _t64(pm), _t64(zm), feed_target=feed)
    assert torch.equal(f1, f2)
    f3, _, _ = TRN.forward(Wt, _t64(mem), lens, _t64(tg2), _t64(pm), _t64(zm))
    assert not torch.equal(f1[:, 2], f3[:, 2])


def test_oracle_masked_losses_by_hand():
    """MaskedMSE divides by the number of nonzero weights (NM·Σ lengths); the masked stop loss is
    TF's weighted cross entropy summed over the mask and divided by its nonzero count."""
    rng = np.random.default_rng(3)
    B, T, NM = 3, 6, 4
    tg, out = rng.normal(size=(B, T, NM)), rng.normal(size=(B, T, NM))
    lens = np.array([6, 2, 4])
    w = (np.arange(T)[None, :] < lens[:, None])
    want = ((out - tg) ** 2 * w[:, :, None]).sum() / (w.sum() * NM)
    assert abs(TRN.masked_mse(_t64(tg), _t64(out), lens).item() - want) < 1e-12
    x, z, q = rng.normal(size=(B, T)) * 3, (rng.random((B, T)) < 0.3).astype(np.float64), 20.0
    l = 1 + (q - 1) * z
    v = w * ((1 - z) * x + l * np.log1p(np.exp(-x)))                  # softplus(-x), textbook form
    got = TRN.masked_stop_loss(_t64(z), _t64(x), lens, q).item()
    assert abs(got - v.sum() / (v != 0).sum()) < 1e-12


def test_oracle_gradients_with_options_match_finite_differences():
    """Free-running steps (gradient through the fed-back frame), masked losses and pos_weight:
    autograd of the restatement against central differences."""
    hp = small_hparams()
    W, mem, lens, tg, st, pm, zm = _case(hp, B=2, T_in=6, T_out=5)
    feed = np.array([1, 0, 1, 0, 0], np.uint8)
    tl = np.array([5, 3])
    pnm = postnet_masks(hp.postnet_num_layers, 2, 5, hp.postnet_channels, seed=1)
    kw = dict(feed_target=feed, target_lengths=tl, pos_weight=7.0)
    _, _, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, reg_weight=1e-3, postnet=True,
                              postnet_masks=pnm, **kw)

    def loss_of(W2):
        names = TRN.train_var_names() + TRN.postnet_var_names()
        Wt = {n: _t64(W2[n]) for n in names}
        fr, sl, _ = TRN.forward(Wt, _t64(mem), lens, _t64(tg), _t64(pm), _t64(zm), feed_target=feed)
        b, s, r = TRN.losses(fr, sl, _t64(tg), _t64(st), Wt, 1e-3, target_lengths=tl, pos_weight=7.0)
        dec = TRN.clip_decoder_output(fr)
        proj, _ = TRN.postnet_train(Wt, dec, _t64(pnm))
        after = TRN.masked_mse(_t64(tg), TRN.clip_decoder_output(dec + proj), tl)
        return float(b + s + r + after)

    rng = np.random.default_rng(5)
    P = "Tacotron_model/inference/"
    for name in [P + "decoder/decoder_prenet/dense_1/kernel", TRN.FP + "kernel", TRN.FP + "bias",
                 TRN.SP + "bias", TRN.L1 + "kernel"]:
        arr = np.asarray(W[name], np.float64)
        for _ in range(3):
            idx = tuple(rng.integers(0, s) for s in arr.shape)
            eps = 1e-6
            Wp, Wm = dict(W), dict(W)
            ap, am = arr.copy(), arr.copy()
            ap[idx] += eps
            am[idx] -= eps
            Wp[name], Wm[name] = ap, am
            fd = (loss_of(Wp) - loss_of(Wm)) / (2 * eps)
            assert abs(fd - g[name][idx]) < 1e-6 + 1e-4 * abs(fd), (name, idx, fd, g[name][idx])


@pytest.mark.gpu
@pytest.mark.parametrize("postnet", [True, False])
def test_gpu_train_teacher_forcing_and_masked_losses(postnet):
    """Free-running steps drawn at ratio 0.5, ragged target lengths under mask_decoder and
    pos_weight 20: frames, losses and every gradient (incl. d memory) against the float64 oracle."""
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(mask_decoder=True, cross_entropy_pos_weight=20.0))
    B, T_in, T_out = 3, 9, 7
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out, seed=29)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=29) if postnet else None
    feed = draw_teacher_forcing(T_out, 0.5, np.random.default_rng(4))
    feed[2], feed[3] = 0, 1                                            # both kinds present
    tl = np.array([T_out, 4, 2], np.int32)
    names = TRN.train_var_names() + (TRN.postnet_var_names() if postnet else [])
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, postnet=postnet)
    try:
        tr.set_step_inputs(targets_lengths=tl, feed_target=feed)
        tr.forward_backward(mem, lens, tg, st, pm, zm, pnm)
        L = tr.losses()
        fr, sl, al = tr.outputs(T_in, T_out)
        grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
        gmem = tr.get("memory", 1, mem.shape)
    finally:
        tr.close()
    out, Lr, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp),
                                 postnet=postnet, postnet_masks=pnm, feed_target=feed, target_lengths=tl,
                                 pos_weight=20.0)
    assert np.abs(fr - out["frames"]).max() < 1e-4
    assert abs(L["before"] - Lr[0]) < 1e-5 * Lr[0] and abs(L["stop_token"] - Lr[1]) < 1e-5 * Lr[1]
    if postnet:
        assert abs(L["after"] - Lr[3]) < 1e-5 * Lr[3]
    for n in names:
        if np.abs(g[n]).max() < 1e-12:
            assert np.abs(grads[n]).max() < 1e-6, n
            continue
        assert _rel(grads[n], g[n]) < 2e-4, (n, _rel(grads[n], g[n]))
    assert _rel(gmem, g["memory"]) < 2e-4


@pytest.mark.gpu
def test_gpu_train_mask_decoder_requires_target_lengths():
    """tacotron.py:56-57: a masked model without target lengths fails the step."""
    from tt2._lib import TT2Error
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(mask_decoder=True))
    W, mem, lens, tg, st, pm, zm = _case(hp, 2, 6, 4)
    tr = TacotronTrainer(hp, W, 2, 6, 4, 0, postnet=False)
    try:
        with pytest.raises(TT2Error, match="targets lengths"):
            tr.forward_backward(mem, lens, tg, st, pm, zm)
        tr.set_step_inputs(targets_lengths=np.array([4, 3]))
        tr.forward_backward(mem, lens, tg, st, pm, zm)
        assert np.isfinite(tr.losses()["loss"])
        with pytest.raises(TT2Error):
            tr.set_step_inputs(targets_lengths=np.array([4, 9]))        # > max_T_out
    finally:
        tr.close()


def test_oracle_smoothing_gradients_match_finite_differences():
    """hp.smoothing in the training graph (attention.py:71-91,150: a = sigmoid(e) / Σ sigmoid(e)
    over the unmasked positions): the restatement's autograd against central differences on the
    attention variables, ragged input lengths."""
    hp = small_hparams()
    W, mem, lens, tg, st, pm, zm = _case(hp, B=2, T_in=6, T_out=4)
    out, _, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, reg_weight=1e-3, smoothing=True)
    al = out["alignments"]
    np.testing.assert_allclose(al.sum(1), 1.0, atol=1e-12)
    assert np.all(al[1, lens[1]:] == 0)

    def loss_of(W2):
        Wt = {n: torch.tensor(np.asarray(W2[n]), dtype=torch.float64) for n in TRN.train_var_names()}
        fr, sl, _ = TRN.forward(Wt, torch.tensor(mem, dtype=torch.float64), lens, torch.tensor(tg, dtype=torch.float64),
                                torch.tensor(pm, dtype=torch.float64), torch.tensor(zm, dtype=torch.float64),
                                smoothing=True)
        b, s, r = TRN.losses(fr, sl, torch.tensor(tg, dtype=torch.float64), torch.tensor(st, dtype=torch.float64),
                             Wt, 1e-3)
        return float(b + s + r)

    rng = np.random.default_rng(2)
    for name in [TRN.LA + "attention_variable_projection", TRN.LA + "attention_bias",
                 TRN.LA + "location_features_convolution/kernel", TRN.P + "decoder/query_layer/kernel"]:
        arr = np.asarray(W[name], np.float64)
        for _ in range(2):
            idx = tuple(rng.integers(0, s) for s in arr.shape)
            eps = 1e-6
            Wp, Wm = dict(W), dict(W)
            ap, am = arr.copy(), arr.copy()
            ap[idx] += eps
            am[idx] -= eps
            Wp[name], Wm[name] = ap, am
            fd = (loss_of(Wp) - loss_of(Wm)) / (2 * eps)
            assert abs(fd - g[name][idx]) < 1e-7 + 1e-4 * abs(fd), (name, idx, fd, g[name][idx])


def test_train_config_smoothing():
    hp = small_hparams()
    hp.override_from_dict(dict(smoothing=True))
    assert train_config(hp, 2, 8, 4).smoothing == 1


@pytest.mark.gpu
def test_gpu_train_smoothing_matches_oracle():
    """hp.smoothing in the training step: the sigmoid normalisation forward (k_tr_ctx) and the
    softmax backward times (1 - sigmoid(e_j)) in the attention backward: fp32 frames / alignments
    within 1e-4 and every gradient (incl. d memory) within 2e-4 of the float64 oracle, with the
    Postnet and ragged lengths; the alignments are not the softmax ones."""
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(smoothing=True))
    B, T_in, T_out = 3, 9, 7
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out, seed=31)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=31)
    names = TRN.train_var_names() + TRN.postnet_var_names()
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, postnet=True)
    try:
        tr.forward_backward(mem, lens, tg, st, pm, zm, pnm)
        L = tr.losses()
        fr, sl, al = tr.outputs(T_in, T_out)
        grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
        gmem = tr.get("memory", 1, mem.shape)
    finally:
        tr.close()
    out, Lr, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp),
                                 postnet=True, postnet_masks=pnm, smoothing=True)
    soft, _, _ = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp))
    assert np.abs(al - soft["alignments"]).max() > 1e-3
    assert np.abs(al - out["alignments"]).max() < 1e-4
    assert np.abs(fr - out["frames"]).max() < 1e-4
    assert abs(L["before"] - Lr[0]) < 1e-5 * Lr[0] and abs(L["after"] - Lr[3]) < 1e-5 * Lr[3]
    for n in names:
        if np.abs(g[n]).max() < 1e-12:
            assert np.abs(grads[n]).max() < 1e-6, n
            continue
        assert _rel(grads[n], g[n]) < 2e-4, (n, _rel(grads[n], g[n]))
    assert _rel(gmem, g["memory"]) < 2e-4


@pytest.mark.gpu
def test_gpu_train_smoothing_fork_widths_bf16():
    """hp.smoothing at the fork widths in the bf16 step: the one-launch attention backward
    (k_tr_att_bwd_q) with the smoothing factor, the persistent forward left out (it keeps the
    softmax): against the float64 oracle at the mixed-precision tolerance of
    test_gpu_train_persistent_forward_close_to_oracle."""
    from tt2.hparams import hparams
    from test_train import _trainer_run
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1, smoothing=True))
    B, T_in, T_out = 4, 37, 10
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    r = _trainer_run(hp, W, (mem, lens, tg, st, pm, zm), {"TT2_TR_PERSIST": "1"})
    assert r["persist"] == 0.0
    out, (b, s, _), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp),
                                        smoothing=True)
    assert np.abs(r["al"] - out["alignments"]).max() < 1e-3
    assert np.abs(r["fr"] - out["frames"]).max() < 1e-2
    assert abs(r["L"]["before"] - b) < 1e-3 * b
    for n in TRN.train_var_names():
        frob = float(np.linalg.norm(r["g"][n] - g[n]) / max(np.linalg.norm(g[n]), 1e-30))
        assert frob < (0.1 if "prenet" in n else 1e-2), (n, frob)
