"""Teacher-forced decoder training step (SURVEY.md §8f rank 1, configs[4]).

CPU: the torch-autograd oracle (oracle/train_ref.py) is pinned to the numpy inference oracle's
teacher-forced decode, its gradients to finite differences, its Adam/clip step to the TF formulas.
GPU (-m gpu): libtt2's training kernels (csrc/train.hip) through the C ABI against that oracle.
Parity unpinned against TF itself.
"""
import numpy as np
import pytest
import torch

from _common import small_hparams
from oracle import tacotron_ref as TR
from oracle import train_ref as TRN
from oracle.hp import oracle_hp
from tt2.synthetic import postnet_masks, prenet_masks, train_batch, zoneout_masks
from tt2.weights import init_tacotron_weights, memory_width

MEM_K = "Tacotron_model/inference/memory_layer/kernel"


def _case(hp, B=3, T_in=9, T_out=7, seed=11):
    W = init_tacotron_weights(hp, seed=5339)
    D = memory_width(hp)
    mem, lens, tg, st = train_batch(B, T_in, T_out, D, seed=seed)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=seed)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=seed)
    return W, mem, lens, tg, st, pm, zm


def test_forward_matches_numpy_inference_oracle():
    """With inference zoneout the torch restatement is the numpy oracle's GTA decode."""
    hp = small_hparams()
    W, mem, lens, tg, st, pm, _ = _case(hp)
    Wt = {n: torch.tensor(np.asarray(W[n]), dtype=torch.float64) for n in TRN.train_var_names()}
    fr, sl, al = TRN.forward(Wt, torch.tensor(mem, dtype=torch.float64), lens,
                             torch.tensor(tg, dtype=torch.float64),
                             torch.tensor(pm, dtype=torch.float64), None,
                             zoneout=hp.tacotron_zoneout_rate)
    mask = (np.arange(mem.shape[1])[None, :] < lens[:, None])
    values = mem.astype(np.float64) * mask[:, :, None]
    keys = values @ np.asarray(W[MEM_K], np.float64)
    ohp = oracle_hp(hp)
    f2, s2, a2 = TR.dynamic_decode(keys, values, lens, W, ohp, pm, tg.shape[1], targets=tg,
                                   dt=np.float64)
    np.testing.assert_allclose(fr.numpy(), f2, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(torch.sigmoid(sl).numpy(), s2, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(al.numpy(), a2, rtol=1e-10, atol=1e-10)


def test_oracle_gradients_match_finite_differences():
    hp = small_hparams()
    W, mem, lens, tg, st, pm, zm = _case(hp, B=2, T_in=6, T_out=4)
    _, _, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, reg_weight=1e-3)
    rng = np.random.default_rng(0)

    def loss_of(W2, mem2):
        Wt = {n: torch.tensor(np.asarray(W2[n]), dtype=torch.float64) for n in TRN.train_var_names()}
        tg_t = torch.tensor(tg, dtype=torch.float64)
        fr, sl, _ = TRN.forward(Wt, torch.tensor(mem2, dtype=torch.float64), lens, tg_t,
                                torch.tensor(pm, dtype=torch.float64),
                                torch.tensor(zm, dtype=torch.float64))
        b, s, r = TRN.losses(fr, sl, tg_t, torch.tensor(st, dtype=torch.float64), Wt, 1e-3)
        return float(b + s + r)

    eps = 1e-6
    for name in (MEM_K, TRN.L1 + "kernel", TRN.LA + "location_features_convolution/kernel",
                 TRN.LA + "attention_variable_projection", TRN.FP + "bias"):
        arr = np.asarray(W[name], np.float64)
        for _ in range(3):
            idx = tuple(rng.integers(0, s) for s in arr.shape)
            Wp, Wm = dict(W), dict(W)
            ap, am = arr.copy(), arr.copy()
            ap[idx] += eps
            am[idx] -= eps
            Wp[name], Wm[name] = ap, am
            fd = (loss_of(Wp, mem.astype(np.float64)) - loss_of(Wm, mem.astype(np.float64))) / (2 * eps)
            assert abs(fd - g[name][idx]) < 1e-6 + 1e-5 * abs(fd), (name, idx, fd, g[name][idx])
    # memory gradient is zero past each row's length (values = memory · mask)
    for b in range(mem.shape[0]):
        assert np.all(g["memory"][b, lens[b]:] == 0)


def test_oracle_postnet_gradients_match_finite_differences():
    """Postnet in training mode (batch-statistics BN, dropout, clipped after loss): autograd of
    the restatement vs central differences on conv, BN and projection variables."""
    hp = small_hparams()
    W, mem, lens, tg, st, pm, zm = _case(hp, B=2, T_in=6, T_out=5)
    pnm = postnet_masks(hp.postnet_num_layers, 2, 5, hp.postnet_channels)
    _, L, g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, 1e-3, postnet=True, postnet_masks=pnm)
    assert len(L) == 4 and L[3] > 0

    def loss_of(W2):
        _, L2, _ = TRN.train_grads(W2, mem, lens, tg, st, pm, zm, 1e-3, postnet=True,
                                   postnet_masks=pnm)
        return sum(L2)

    rng = np.random.default_rng(1)
    eps = 1e-6
    for name in (TRN.PN.format(1) + "conv1d/kernel", TRN.PN.format(3) + "batch_normalization/gamma",
                 TRN.PN.format(5) + "batch_normalization/beta", TRN.PP + "kernel",
                 TRN.L2 + "kernel"):
        arr = np.asarray(W[name], np.float64)
        for _ in range(2):
            idx = tuple(rng.integers(0, n) for n in arr.shape)
            Wp, Wm = dict(W), dict(W)
            ap, am = arr.copy(), arr.copy()
            ap[idx] += eps
            am[idx] -= eps
            Wp[name], Wm[name] = ap, am
            fd = (loss_of(Wp) - loss_of(Wm)) / (2 * eps)
            assert abs(fd - g[name][idx]) < 1e-6 + 1e-5 * abs(fd), (name, idx, fd, g[name][idx])


def test_learning_rate_and_adam_formulas():
    hp = small_hparams()
    assert TRN.learning_rate(0, hp) == hp.tacotron_initial_learning_rate
    lr = TRN.learning_rate(hp.tacotron_start_decay + hp.tacotron_decay_steps, hp)
    assert abs(lr - max(hp.tacotron_initial_learning_rate * hp.tacotron_decay_rate,
                        hp.tacotron_final_learning_rate)) < 1e-15
    assert TRN.learning_rate(10 ** 7, hp) == hp.tacotron_final_learning_rate
    p = {"w": np.array([1.0, -2.0])}
    g = {"w": np.array([3.0, 4.0])}                     # global norm 5 -> clipped to 1
    m = {"w": np.zeros(2)}
    v = {"w": np.zeros(2)}
    gn = TRN.clip_and_adam(p, g, m, v, 1, 1e-3)
    assert gn == 5.0
    # first Adam step moves each weight by ~lr·sign(g)
    np.testing.assert_allclose(p["w"], [1.0 - 1e-3, -2.0 - 1e-3], rtol=0, atol=1e-7)


# ---------------------------------------------------------------------------------------------
# GPU parity (C ABI) against the float64 oracle
# ---------------------------------------------------------------------------------------------
def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _clip(hp):
    lo, hi = (-hp.max_abs_value, hp.max_abs_value) if hp.symmetric_mels else (0.0, hp.max_abs_value)
    return (lo - hp.lower_bound_decay, hi) if hp.clip_outputs else None


def _gpu_vs_oracle(hp, B, T_in, T_out, use_zoneout_masks=True, seed=11):
    from tt2.train import TacotronTrainer
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out, seed)
    if not use_zoneout_masks:
        zm = None
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, postnet=False)
    try:
        tr.forward_backward(mem, lens, tg, st, pm, zm)
        L = tr.losses()
        fr, sl, al = tr.outputs(T_in, T_out)
        grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in TRN.train_var_names()}
        gmem = tr.get("memory", 1, mem.shape)
    finally:
        tr.close()
    out, (b, s, r), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight,
                                        clip=_clip(hp))
    return (fr, sl, al, L, grads, gmem), (out, (b, s, r), g)


@pytest.mark.gpu
@pytest.mark.parametrize("zoneout_masks", [True, False])
def test_gpu_train_forward_backward_small(zoneout_masks):
    """Small widths, ragged lengths: outputs 1e-4 (north_star's mel tolerance), losses 1e-5
    relative, every gradient within 1e-4 of the float64 oracle relative to its max."""
    hp = small_hparams()
    (fr, sl, al, L, grads, gmem), (out, (b, s, r), g) = _gpu_vs_oracle(hp, 3, 9, 12, zoneout_masks)
    assert np.abs(fr - out["frames"]).max() < 1e-4
    assert np.abs(sl - out["stop_logits"]).max() < 1e-4
    assert np.abs(al - out["alignments"]).max() < 1e-5
    assert abs(L["before"] - b) < 1e-5 * abs(b) + 1e-7
    assert abs(L["stop_token"] - s) < 1e-5 * abs(s) + 1e-7
    assert abs(L["regularization"] - r) < 1e-4 * abs(r) + 1e-9
    for n in TRN.train_var_names():
        assert _rel(grads[n], g[n]) < 1e-4, (n, _rel(grads[n], g[n]))
    assert _rel(gmem, g["memory"]) < 1e-4
    for bb in range(3):
        assert np.all(gmem[bb, _case(hp, 3, 9, 12)[2][bb]:] == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T_in,T_out", [(1, 5, 1), (1, 17, 9), (5, 16, 3)])
def test_gpu_train_edge_shapes(B, T_in, T_out):
    """Single-row batches, a one-step decode, T_in on a 16-row attention-tile boundary, with the
    Postnet: outputs, losses and every gradient against the oracle."""
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out, seed=23)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=23)
    names = TRN.train_var_names() + TRN.postnet_var_names()
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0)
    try:
        tr.forward_backward(mem, lens, tg, st, pm, zm, pnm)
        L = tr.losses()
        fr, sl, al = tr.outputs(T_in, T_out)
        grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
    finally:
        tr.close()
    out, (b, s, r, after), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight,
                                               clip=_clip(hp), postnet=True, postnet_masks=pnm)
    assert np.abs(fr - out["frames"]).max() < 1e-4
    assert np.abs(al - out["alignments"]).max() < 1e-5
    assert abs(L["before"] - b) < 1e-5 * b and abs(L["after"] - after) < 1e-5 * after
    for n in names:
        if np.abs(g[n]).max() < 1e-12:
            assert np.abs(grads[n]).max() < 1e-6, n
            continue
        assert _rel(grads[n], g[n]) < 2e-4, (n, _rel(grads[n], g[n]))


@pytest.mark.gpu
def test_gpu_train_clipped_decoder_output():
    """clip_outputs with a tight range (max_abs_value 0.02): decoder_output is clipped before the
    before-loss (tacotron.py:360-361) and no gradient flows through clipped frames."""
    hp = small_hparams()
    hp.override_from_dict(dict(max_abs_value=0.02, lower_bound_decay=0.01))
    (fr, sl, al, L, grads, gmem), (out, (b, s, r), g) = _gpu_vs_oracle(hp, 3, 9, 12)
    assert np.mean(np.abs(fr) >= 0.02 - 1e-7) > 0.1            # the clip is active
    assert np.abs(fr - out["frames"]).max() < 1e-5
    assert abs(L["before"] - b) < 1e-5 * abs(b)
    for n in TRN.train_var_names():
        assert _rel(grads[n], g[n]) < 1e-4, (n, _rel(grads[n], g[n]))


@pytest.mark.gpu
def test_gpu_train_forward_backward_full_widths():
    """Fork-default widths (D_mem 1024, LSTM 1024, attention 128/32/31, prenet 256) on a short
    ragged batch: the production kernel shapes (A = 128 → 2 sub-rows per attention block)."""
    hp = small_hparams()
    hp.override_from_dict(dict(attention_dim=128, attention_filters=32, prenet_layers=[256, 256],
                               decoder_lstm_units=1024, embedding_dim=512, enc_conv_channels=512,
                               encoder_lstm_units=256, style_embed_depth=256, style_att_dim=128,
                               reference_filters=[32, 32, 64, 64, 128, 128], reference_depth=128))
    (fr, sl, al, L, grads, gmem), (out, (b, s, r), g) = _gpu_vs_oracle(hp, 4, 37, 10)
    assert np.abs(fr - out["frames"]).max() < 1e-4
    assert np.abs(al - out["alignments"]).max() < 1e-5
    assert abs(L["before"] - b) < 1e-5 * abs(b)
    for n in TRN.train_var_names():
        assert _rel(grads[n], g[n]) < 2e-4, (n, _rel(grads[n], g[n]))
    assert _rel(gmem, g["memory"]) < 2e-4


@pytest.mark.gpu
def test_gpu_train_adam_updates_match_oracle():
    """Two steps of clip_by_global_norm + Adam against oracle/train_ref.clip_and_adam."""
    from tt2.train import TacotronTrainer, learning_rate
    hp = small_hparams()
    B, T_in, T_out = 2, 8, 6
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    names = TRN.train_var_names()
    p = {n: np.asarray(W[n], np.float64) for n in names}
    m = {n: np.zeros_like(p[n]) for n in names}
    v = {n: np.zeros_like(p[n]) for n in names}
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, postnet=False)
    try:
        for step in (1, 2):
            tr.forward_backward(mem, lens, tg, st, pm, zm)
            lr = tr.apply(step)
            L = tr.losses()
            Wcur = dict(W)
            Wcur.update(p)
            _, _, g = TRN.train_grads(Wcur, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight)
            g.pop("memory")
            gn = TRN.clip_and_adam(p, g, m, v, step, learning_rate(step - 1, hp))
            assert abs(L["grad_norm"] - gn) < 1e-4 * gn
            assert lr == learning_rate(step - 1, hp)
            for n in names:
                got = tr.get(n, 0, p[n].shape)
                assert np.abs(got - p[n]).max() < 1e-6 + 1e-5 * np.abs(p[n]).max(), n
    finally:
        tr.close()


@pytest.mark.gpu
def test_gpu_train_bf16_gemms_close_to_oracle():
    """configs[4]'s bf16 mode (bf16 GEMM operands, fp32 accumulation / state / optimizer) against
    the float64 oracle at fork-default widths: a mixed-precision tolerance, not parity."""
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(attention_dim=128, attention_filters=32, prenet_layers=[256, 256],
                               decoder_lstm_units=1024))
    B, T_in, T_out = 4, 37, 10
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", postnet=False)
    try:
        tr.forward_backward(mem, lens, tg, st, pm, zm)
        L = tr.losses()
        fr, sl, al = tr.outputs(T_in, T_out)
        grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in TRN.train_var_names()}
    finally:
        tr.close()
    out, (b, s, r), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight,
                                        clip=_clip(hp))
    errs = {n: _rel(grads[n], g[n]) for n in TRN.train_var_names()}
    frob = {n: float(np.linalg.norm(grads[n] - g[n]) / max(np.linalg.norm(g[n]), 1e-30))
            for n in TRN.train_var_names()}
    for n in TRN.train_var_names():
        print("  {:90s} maxrel {:.3e} frob {:.3e}".format(n, errs[n], frob[n]))
    print("bf16 frames max|err| {:.3e}, loss rel {:.3e}, worst grad {}".format(
        float(np.abs(fr - out["frames"]).max()), abs(L["before"] - b) / b,
        max(errs.items(), key=lambda kv: kv[1])))
    assert np.abs(fr - out["frames"]).max() < 1e-2
    assert abs(L["before"] - b) < 1e-3 * b
    for n, e in errs.items():
        if "prenet" in n:
            # bf16-rounded prenet pre-activations near 0 flip ReLU/keep decisions; over the 40
            # rows of this case one flip moves a whole row's contribution (measured 2-6 %)
            assert frob[n] < 0.1, (n, frob[n])
        else:
            assert e < 1e-2, (n, e)  # measured 0.2-0.5 % (bf16 operand rounding)


@pytest.mark.gpu
@pytest.mark.parametrize("dropout", [True, False])
def test_gpu_train_with_postnet(dropout):
    """Decoder + Postnet training step (tacotron.py:362-381): training-mode batch norm, Postnet
    dropout keep bits, after loss on the clipped mel; every gradient (decoder, Postnet convs, BN
    gamma/beta, projection) and d memory against the float64 oracle, then apply() moves the BN
    moving averages by (1 - 0.99)·(batch - moving) (UPDATE_OPS)."""
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    B, T_in, T_out = 3, 9, 12
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels) if dropout else None
    names = TRN.train_var_names() + TRN.postnet_var_names()
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0)
    try:
        tr.forward_backward(mem, lens, tg, st, pm, zm, pnm)
        L = tr.losses()
        grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
        gmem = tr.get("memory", 1, mem.shape)
        tr.apply(1)
        tr.losses()
        moving = {n: tr.get(n, 0, np.asarray(W[n]).shape) for n in TRN.postnet_stat_names()}
    finally:
        tr.close()
    out, (b, s, r, after), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm,
                                               hp.tacotron_reg_weight, clip=_clip(hp),
                                               postnet=True, postnet_masks=pnm)
    assert abs(L["before"] - b) < 1e-5 * b
    assert abs(L["after"] - after) < 1e-5 * after, (L["after"], after)
    assert abs(L["regularization"] - r) < 1e-4 * r
    for n in names:
        if np.abs(g[n]).max() < 1e-12:
            # the last conv's bias feeds batch-statistics BN directly (no tanh): its gradient is
            # exactly zero in exact arithmetic, fp32 leaves rounding noise
            assert np.abs(grads[n]).max() < 1e-6, n
            continue
        assert _rel(grads[n], g[n]) < 2e-4, (n, _rel(grads[n], g[n]))
    assert _rel(gmem, g["memory"]) < 2e-4
    for i, (bm, bv) in enumerate(out["bn_stats"]):
        mn, vn = TRN.postnet_stat_names()[2 * i: 2 * i + 2]
        np.testing.assert_allclose(moving[mn], TRN.bn_moving_update(np.asarray(W[mn], np.float64), bm),
                                   rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(moving[vn], TRN.bn_moving_update(np.asarray(W[vn], np.float64), bv),
                                   rtol=1e-5, atol=1e-6)


def test_train_config_validation_without_gpu():
    """The C ABI rejects shapes the training kernels' LDS tiles cannot hold before touching the
    device (no GPU needed): max_T_in > 320, attention_dim not dividing 256, memory_dim > 1024."""
    import ctypes
    from tt2 import _lib
    from tt2.train import train_config
    lib = _lib.load_library()
    hp = small_hparams()

    def create_fails(cfg, msg):
        h = ctypes.c_void_p()
        assert lib.tt2_train_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -1
        assert msg in lib.tt2_last_error().decode()

    create_fails(train_config(hp, 2, 400, 8), "max_T_in")
    cfg = train_config(hp, 2, 16, 8)
    cfg.attention_dim = 48
    create_fails(cfg, "attention_dim")
    cfg = train_config(hp, 2, 16, 8)
    cfg.memory_dim = 2048
    create_fails(cfg, "memory_dim")


@pytest.mark.gpu
def test_gpu_train_full_size_properties():
    """configs[4] shape (B=64, T_in=150, T_out=800, fork-default widths, Postnet): too large for the
    float64 oracle, so size-independent properties -- fp32 and bf16 agree on the losses (1e-3
    relative) and gradient norm (2 %), everything finite, and three clipped-Adam steps on one
    batch lower the total loss."""
    from tt2.hparams import hparams
    from tt2.train import TacotronTrainer
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    B, T_in, T_out = 64, 150, 800
    W = init_tacotron_weights(hp, seed=5339)
    mem, lens, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=7)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=7)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=7)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=7)
    res = {}
    for prec in ("fp32", "bf16"):
        tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision=prec)
        try:
            losses = []
            for step in (1, 2, 3):
                tr.forward_backward(mem, lens, tg, st, pm, zm, pnm)
                tr.apply(step)
                losses.append(tr.losses())
            g = tr.get(TRN.L1 + "kernel", 0, np.asarray(W[TRN.L1 + "kernel"]).shape)
        finally:
            tr.close()
        assert all(np.isfinite([L["loss"], L["grad_norm"]]).all() for L in losses)
        assert np.isfinite(g).all()
        assert losses[-1]["loss"] < losses[0]["loss"], [L["loss"] for L in losses]
        res[prec] = losses
    for k in ("before", "after", "stop_token"):
        a, b = res["fp32"][0][k], res["bf16"][0][k]
        assert abs(a - b) < 1e-3 * abs(a), (k, a, b)
    a, b = res["fp32"][0]["grad_norm"], res["bf16"][0]["grad_norm"]
    assert abs(a - b) < 2e-2 * a, (a, b)


def test_frontend_oracle_inference_mode_matches_numpy_oracle():
    """The torch front-end restatement with moving BN statistics and no masks IS the inference
    graph: its memory equals oracle/tacotron_ref.py's encoder + style path (pins the restatement
    the front-end gradients come from)."""
    import torch
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    from tt2.synthetic import tacotron_inputs
    ids, lens, re, rs = tacotron_inputs(3, 9, 70, seed=4)
    Wt = {n: torch.tensor(np.asarray(W[n]), dtype=torch.float64) for n in TRN.frontend_var_names()}
    mem, _ = TRN.frontend_forward(Wt, ids, lens, re, rs, moving=W)
    oh = oracle_hp(hp)
    enc = TR.encoder(ids, lens, W, oh, np.float64)
    st = TR.style_embedding(re, rs, W, oh, np.float64)
    mask = (np.arange(9)[None] < lens[:, None])[..., None]
    want = np.concatenate([enc, np.broadcast_to(st[:, None], (3, 9, st.shape[1]))], -1)
    np.testing.assert_allclose(mem.numpy() * mask, want * mask, rtol=0, atol=1e-9)


def _front_case(hp, B=3, T_in=9, T_out=6, T_ref=70, seed=32, masks=True):
    from tt2.synthetic import enc_conv_masks, enc_zoneout_masks, tacotron_inputs
    W = init_tacotron_weights(hp, seed=5339)
    ids, lens, re, rs = tacotron_inputs(B, T_in, T_ref, seed=seed)
    _, _, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=seed)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=seed)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=seed)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=seed)
    em = enc_conv_masks(hp.enc_conv_num_layers, B, T_in, hp.enc_conv_channels, seed=seed) if masks else None
    ezm = enc_zoneout_masks(T_in, B, hp.encoder_lstm_units, seed=seed) if masks else None
    return W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm


def test_frontend_oracle_gradients_match_finite_differences():
    """Spot-check the front-end autograd (embedding, encoder conv / BN / dropout, BiLSTM with
    training zoneout and lengths, refnet conv2d / BN / GRU / dense, GST) with central differences."""
    hp = small_hparams()
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, B=2, T_in=6, T_out=3, T_ref=40)
    _, g, _ = TRN.train_grads_frontend(W, ids, lens, re, rs, tg, st, pm, zm, em, ezm, reg_weight=1e-3,
                                       postnet_masks=pnm)

    def loss_of(W2):
        names = TRN.frontend_var_names() + TRN.train_var_names() + TRN.postnet_var_names()
        Wt = {n: torch.tensor(np.asarray(W2[n]), dtype=torch.float64) for n in names}
        mem, _ = TRN.frontend_forward(Wt, ids, lens, re, rs, em, ezm)
        tg_t = torch.tensor(tg, dtype=torch.float64)
        fr, sl, _ = TRN.forward(Wt, mem, lens, tg_t, torch.tensor(pm, dtype=torch.float64),
                                torch.tensor(zm, dtype=torch.float64))
        b, s, r = TRN.losses(fr, sl, tg_t, torch.tensor(st, dtype=torch.float64), Wt, 1e-3)
        dec = TRN.clip_decoder_output(fr)
        proj, _ = TRN.postnet_train(Wt, dec, torch.tensor(pnm, dtype=torch.float64))
        after = ((TRN.clip_decoder_output(dec + proj) - tg_t) ** 2).mean()
        return float(b + s + r + after)

    rng = np.random.default_rng(3)
    P = "Tacotron_model/inference/"
    for name in [P + "inputs_embedding",
                 P + "encoder_convolutions/conv_layer_2_encoder_convolutions/conv1d/kernel",
                 P + "encoder_convolutions/conv_layer_1_encoder_convolutions/batch_normalization/gamma",
                 P + "encoder_LSTM/bidirectional_rnn/bw/lstm_cell/kernel",
                 P + "refnet_emt/conv2d_1/conv2d/kernel", P + "refnet_spk/rnn/gru_cell/gates/kernel",
                 P + "refnet_emt/dense/kernel", P + "style_tokens_spk",
                 P + "Multihead-attention-emt/attention_v", P + "Multihead-attention-spk/attention_g"]:
        w = np.asarray(W[name], np.float64)
        idx = np.unravel_index(np.argmax(np.abs(g[name])), w.shape) if w.ndim else ()
        eps = 1e-5
        Wp, Wm = dict(W), dict(W)
        wp, wm = w.copy(), w.copy()
        wp[idx] += eps
        wm[idx] -= eps
        Wp[name], Wm[name] = wp, wm
        fd = (loss_of(Wp) - loss_of(Wm)) / (2 * eps)
        assert abs(fd - g[name][idx]) < 1e-5 + 1e-4 * abs(fd), (name, fd, g[name][idx])


def _relu_margin(W, ids, re, rs, em):
    """Smallest |pre-activation| of every front-end ReLU (encoder convs; refnet BN outputs) in
    float64: below ~1e-6 an fp32 device run may take the other side of the kink than the float64
    oracle, and one flipped element moves a batch-norm parameter's gradient by percents."""
    P = "Tacotron_model/inference/"
    Wt = {n: torch.tensor(np.asarray(W[n]), dtype=torch.float64) for n in TRN.frontend_var_names()}
    m = np.inf
    for tag, ref in (("emt", re), ("spk", rs)):
        r = TRN.RN.format(tag)
        h = torch.as_tensor(ref, dtype=torch.float64)[..., None]
        for i in range(6):
            s = r + "conv2d_{}/".format(i)
            a = TRN._conv2d_same_s2(h, Wt[s + "conv2d/kernel"], Wt[s + "conv2d/bias"])
            y, _ = TRN._bn_train(a, Wt[s + "batch_normalization/gamma"],
                                 Wt[s + "batch_normalization/beta"], (0, 1, 2))
            m = min(m, float(y.abs().min()))
            h = torch.relu(y)
    x = Wt[P + "inputs_embedding"][torch.as_tensor(ids).long()]
    for i in range(1, 4):
        s = TRN.EC.format(i)
        k = Wt[s + "conv1d/kernel"]
        pad = (k.shape[0] - 1) // 2
        xp = torch.nn.functional.pad(x, (0, 0, pad, k.shape[0] - 1 - pad))
        z = torch.einsum("btck,kcn->btn", xp.unfold(1, k.shape[0], 1), k) + Wt[s + "conv1d/bias"]
        m = min(m, float(z.abs().min()))
        y, _ = TRN._bn_train(torch.relu(z), Wt[s + "batch_normalization/gamma"],
                             Wt[s + "batch_normalization/beta"], (0, 1))
        x = y if em is None else y / 0.5 * torch.as_tensor(em[i - 1], dtype=torch.float64)
    return m


@pytest.mark.parametrize("masks", [True, False])
def test_frontend_case_has_relu_margin(masks):
    """The GPU front-end parity case keeps every ReLU input >= 1e-5 away from the kink."""
    hp = small_hparams()
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, masks=masks)
    assert _relu_margin(W, ids, re, rs, em) > 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("masks", [True, False])
def test_gpu_train_frontend_matches_oracle(masks):
    """The whole configs[4] step from ids + reference mels (tt2_train_forward_backward_text_dev):
    every front-end, decoder and Postnet gradient within 2e-4 (relative to its max) of the torch
    float64 oracle, the losses, and the front-end BN moving averages after apply."""
    from tt2.train import TacotronTrainer, init_style_disc_weights
    hp = small_hparams()
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, masks=masks)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    # the default graph's style-embedding losses (tacotron.py:486-495, 812-846): orthogonality
    # always (hp default), the classifiers in the masked case (labels incl. an out-of-range one)
    n_emt, n_spk = (4, 3) if masks else (0, 0)
    W.update(init_style_disc_weights(hp, n_emt, n_spk, seed=3))
    el, sl = np.array([1, 3, 0], np.int32), np.array([2, 0, 7], np.int32)
    style = dict(emt_labels=el, spk_labels=sl, n_emt=n_emt, n_spk=n_spk, orthog_weight=0.02)
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1], n_emt=n_emt, n_spk=n_spk)
    try:
        if masks:
            tr.set_style_labels(el, sl)
        tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
        L = tr.losses()
        (b, s_, r, a, le, ls, lo), g, stats = TRN.train_grads_frontend(
            W, ids, lens, re, rs, tg, st, pm, zm, em, ezm, hp.tacotron_reg_weight, postnet_masks=pnm, style=style)
        assert abs(L["before"] - b) < 1e-4 * b and abs(L["after"] - a) < 1e-4 * a
        assert abs(L["regularization"] - r) < 1e-4 * r + 1e-12
        assert abs(L["style_emb_orthog_loss"] - lo) < 1e-4 * lo and lo > 0
        assert abs(L["style_emb_loss_emt"] - le) < 1e-4 * max(le, 1e-3) and abs(L["style_emb_loss_spk"] - ls) < 1e-4 * max(ls, 1e-3)
        assert (le > 0) == bool(masks)
        for n in (TRN.frontend_var_names() + TRN.style_disc_var_names(False, n_emt, n_spk) + TRN.train_var_names()
                  + TRN.postnet_var_names()):
            got = tr.get(n, 1, np.asarray(W[n]).shape)
            if np.abs(g[n]).max() < 1e-12:   # a conv bias feeding batch-statistics BN: exactly 0
                assert np.abs(got).max() < 1e-6, (n, np.abs(got).max())
                continue
            assert _rel(got, g[n]) < 2e-4, (n, _rel(got, g[n]))
        tr.apply(1)
        P = "Tacotron_model/inference/"
        scopes = ["encoder_convolutions/conv_layer_{}_encoder_convolutions/".format(i) for i in (1, 2, 3)]
        scopes += ["refnet_{}/conv2d_{}/".format(t, i) for t in ("emt", "spk") for i in range(6)]
        for sc, (mean, var) in zip(scopes, stats):
            mm = tr.get(P + sc + "batch_normalization/moving_mean", 0, mean.shape)
            want = TRN.bn_moving_update(np.asarray(W[P + sc + "batch_normalization/moving_mean"], np.float64), mean)
            np.testing.assert_allclose(mm, want, rtol=1e-5, atol=1e-5, err_msg=sc)
    finally:
        tr.close()


@pytest.mark.gpu
def test_gpu_train_bf16_library_gemms_match_kernels():
    """bf16 mode routes the large plain products (weight gradients over all T·B rows, >= 2e10
    flops) through the 256 x 256 x 64 LDS-DMA bf16 kernel (gemm.h gemm_bf16_kc: padded K-contiguous
    bf16 copies, K split over work-groups) after the same bf16 operand rounding; TT2_TRAIN_BLAS=0
    keeps them on gemm_x3_kernel.  Same inputs, fork-default widths, T·B = 2000 rows (K not a
    multiple of the 64-deep step, M not of the 256-row tile): the forward, the losses and d memory
    are identical (those products only produce terminal weight gradients), every gradient agrees
    to fp32 accumulation-order level, and the context counts the large-product calls."""
    import os
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(attention_dim=128, attention_filters=32, prenet_layers=[256, 256],
                               decoder_lstm_units=1024))
    B, T_in, T_out = 8, 40, 250
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    names = TRN.train_var_names()
    res = {}
    old = os.environ.get("TT2_TRAIN_BLAS")
    try:
        for flag in ("1", "0"):
            os.environ["TT2_TRAIN_BLAS"] = flag
            tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", postnet=False)
            try:
                tr.forward_backward(mem, lens, tg, st, pm, zm)
                L = tr.losses()
                grads = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
                gmem = tr.get("memory", 1, mem.shape)
                nblas = int(tr.get("diag:blas_calls", 0, (1,))[0])
            finally:
                tr.close()
            res[flag] = (L, grads, gmem)
            # on: the two LSTM kernel gradients (2e10+ flops each at T·B = 2000); off: none
            assert nblas == (2 if flag == "1" else 0), (flag, nblas)
    finally:
        if old is None:
            os.environ.pop("TT2_TRAIN_BLAS", None)
        else:
            os.environ["TT2_TRAIN_BLAS"] = old
    (La, ga, ma), (Lb, gb, mb) = res["1"], res["0"]
    assert La["before"] == Lb["before"] and La["stop_token"] == Lb["stop_token"]
    np.testing.assert_array_equal(ma, mb)
    for n in names:
        frob = float(np.linalg.norm(ga[n] - gb[n]) / max(np.linalg.norm(gb[n]), 1e-30))
        assert frob < 1e-4, (n, frob)


@pytest.mark.gpu
def test_gpu_train_fused_lstm_matches_split_k_path():
    """k_tr_fused (each per-step LSTM product with its consumer's epilogue in one launch, forward
    and backward, on bf16 row shadows) against the split-K products + combines (TT2_TR_FUSED=0) on
    the same bf16 step at fork widths: same operand rounding rule, different fp32 summation order.
    The order moves activations by ~1e-7, which occasionally flips the bf16 rounding of a later
    operand (2^-8 relative), so the gradients agree to bf16-rounding level, not bit for bit: losses
    within 1e-5 relative, every gradient within 1e-2 (Frobenius, relative; measured <= 3e-3 for the
    prenet kernels, the most sensitive; a wrong column or row would be O(1))."""
    import os
    from tt2.hparams import hparams
    from tt2.train import TacotronTrainer
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    B, T_in, T_out = 16, 40, 24
    W = init_tacotron_weights(hp, seed=5339)
    mem, lens, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=3)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=3)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=3)
    res = {}
    for mode in ("1", "0"):
        old = os.environ.get("TT2_TR_FUSED")
        os.environ["TT2_TR_FUSED"] = mode
        try:
            tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", postnet=False)
            try:
                tr.forward_backward(mem, lens, tg, st, pm, zm)
                L = tr.losses()
                g = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in TRN.train_var_names()}
            finally:
                tr.close()
        finally:
            if old is None:
                del os.environ["TT2_TR_FUSED"]
            else:
                os.environ["TT2_TR_FUSED"] = old
        res[mode] = (L, g)
    (La, ga), (Lb, gb) = res["1"], res["0"]
    for k in ("before", "stop_token"):
        assert abs(La[k] - Lb[k]) < 1e-5 * abs(Lb[k]), (k, La[k], Lb[k])
    for n in ga:
        rel = float(np.linalg.norm(ga[n] - gb[n]) / max(np.linalg.norm(gb[n]), 1e-30))
        print("  {:90s} rel {:.3e}".format(n, rel))
        assert rel < 1e-2, (n, rel)


@pytest.mark.gpu
def test_gpu_train_frontend_without_gst_matches_oracle():
    """hp.use_gst = False (tacotron.py:284-291): the 128-wide reference embeddings are the style
    embeddings (no style tokens, no style attention; D_mem = 2U + 2·128).  The whole step from ids
    + reference mels against the torch float64 oracle: losses and every gradient within 2e-4."""
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(use_gst=False))
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, masks=True)
    assert memory_width(hp) == 2 * hp.encoder_lstm_units + 256
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1])
    try:
        tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
        L = tr.losses()
        # the default graph's orthogonality loss on the two reference embeddings (hp default on)
        style = dict(emt_labels=None, spk_labels=None, n_emt=0, n_spk=0, orthog_weight=0.02)
        (b, s_, r, a, le, ls, lo), g, _ = TRN.train_grads_frontend(
            W, ids, lens, re, rs, tg, st, pm, zm, em, ezm, hp.tacotron_reg_weight, postnet_masks=pnm,
            style=style, use_gst=False)
        assert abs(L["before"] - b) < 1e-4 * b and abs(L["after"] - a) < 1e-4 * a
        assert abs(L["style_emb_orthog_loss"] - lo) < 1e-4 * lo and lo > 0
        names = TRN.frontend_var_names(use_gst=False) + TRN.train_var_names() + TRN.postnet_var_names()
        assert not any("style_tokens" in n or "Multihead" in n for n in names)
        for n in names:
            got = tr.get(n, 1, np.asarray(W[n]).shape)
            if np.abs(g[n]).max() < 1e-12:   # a conv bias feeding batch-statistics BN: exactly 0
                assert np.abs(got).max() < 1e-6, (n, np.abs(got).max())
                continue
            assert _rel(got, g[n]) < 2e-4, (n, _rel(got, g[n]))
    finally:
        tr.close()


def _adain_case(hp, B=3, T_in=9, T_out=6, T_ref=40, seed=33):
    from tt2.synthetic import enc_conv_masks, enc_zoneout_masks, tacotron_inputs
    W = init_tacotron_weights(hp, seed=5339, style="adain")
    ids, lens, re, rs = tacotron_inputs(B, T_in, T_ref, seed=seed)
    _, _, tg, st = train_batch(B, T_in, T_out, memory_width(hp, style="adain"), seed=seed)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=seed)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=seed)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=seed)
    em = enc_conv_masks(hp.enc_conv_num_layers, B, T_in, hp.enc_conv_channels, seed=seed)
    ezm = enc_zoneout_masks(T_in, B, hp.encoder_lstm_units, seed=seed)
    return W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm


def test_adain_oracle_gradients_match_finite_differences():
    """The AdaIN front end of the training oracle (ReferenceEncoderAdaIn, modules.py:66-107: two conv
    stacks without BN, the moments restyle, GRU + dense) against central differences on the refnet
    variables of both stacks, the GRU and the dense."""
    hp = small_hparams()
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _adain_case(hp, B=2, T_in=6, T_out=3, T_ref=24)
    _, g, _ = TRN.train_grads_frontend(W, ids, lens, re, rs, tg, st, pm, zm, em, ezm, reg_weight=1e-3,
                                       postnet_masks=pnm, adain=True)
    names = TRN.frontend_var_names(adain=True) + TRN.train_var_names() + TRN.postnet_var_names()
    assert "Tacotron_model/inference/refnet/conv2d_3/conv2d_1/kernel" in names

    def loss_of(W2):
        Wt = {n: torch.tensor(np.asarray(W2[n]), dtype=torch.float64) for n in names}
        mem, _ = TRN.frontend_forward(Wt, ids, lens, re, rs, em, ezm, adain=True)
        tg_t = torch.tensor(tg, dtype=torch.float64)
        fr, sl, _ = TRN.forward(Wt, mem, lens, tg_t, torch.tensor(pm, dtype=torch.float64),
                                torch.tensor(zm, dtype=torch.float64))
        b, s, r = TRN.losses(fr, sl, tg_t, torch.tensor(st, dtype=torch.float64), Wt, 1e-3)
        dec = TRN.clip_decoder_output(fr)
        proj, _ = TRN.postnet_train(Wt, dec, torch.tensor(pnm, dtype=torch.float64))
        mel = TRN.clip_decoder_output(dec + proj)
        return float(b + s + r + ((mel - tg_t) ** 2).mean())

    rng = np.random.default_rng(3)
    P = "Tacotron_model/inference/refnet/"
    for n in (P + "conv2d_0/conv2d/kernel", P + "conv2d_3/conv2d_1/kernel", P + "conv2d_5/conv2d_1/bias",
              P + "conv2d_4/conv2d/bias", P + "rnn/gru_cell/gates/kernel", P + "dense/kernel"):
        W64 = {k: np.asarray(v, np.float64) for k, v in W.items()}
        idx = np.unravel_index(np.argmax(np.abs(g[n])), np.shape(W64[n]))
        h = 1e-6
        Wp, Wm = dict(W64), dict(W64)
        Wp[n] = W64[n].copy(); Wp[n][idx] += h
        Wm[n] = W64[n].copy(); Wm[n][idx] -= h
        fd = (loss_of(Wp) - loss_of(Wm)) / (2 * h)
        assert abs(fd - g[n][idx]) <= 1e-6 + 1e-4 * abs(fd), (n, fd, g[n][idx])


@pytest.mark.gpu
def test_gpu_train_frontend_adain_matches_oracle():
    """args.adain (tacotron.py:236-242, 266-268; modules.py:66-107) in training: speaker and emotion
    conv stacks without batch norm (strides (2,2),(2,2),(1,1)x4), the speaker map restyled by the
    emotion map's moments, GRU + dense tanh as the 128-wide style embedding, backward through the
    restyle into both stacks.  fp32: the whole step from ids + reference mels against the torch
    float64 oracle, losses and every gradient within 2e-4.  bf16 GEMM operands (configs[4]'s mode):
    losses within 1e-2 of fp32 and the front-end gradient direction (cosine) above 0.97 -- single
    gradients of a bf16 step move by ReLU / dropout-boundary flips, as in the other bf16 tests."""
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _adain_case(hp)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    names = TRN.frontend_var_names(adain=True) + TRN.train_var_names() + TRN.postnet_var_names()
    fe = TRN.frontend_var_names(adain=True)
    res = {}
    for precision in ("fp32", "bf16"):
        tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1], precision=precision,
                             style="adain")
        try:
            tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
            res[precision] = (tr.losses(), {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names})
        finally:
            tr.close()
    L, got = res["fp32"]
    (b, s_, r, a), g, _ = TRN.train_grads_frontend(
        W, ids, lens, re, rs, tg, st, pm, zm, em, ezm, hp.tacotron_reg_weight, postnet_masks=pnm, adain=True)
    assert abs(L["before"] - b) < 2e-4 * b and abs(L["after"] - a) < 2e-4 * a
    for n in names:
        if np.abs(g[n]).max() < 1e-12:   # a conv bias feeding batch-statistics BN: exactly 0
            assert np.abs(got[n]).max() < 1e-6, (n, np.abs(got[n]).max())
            continue
        assert _rel(got[n], g[n]) < 2e-4, (n, _rel(got[n], g[n]))
    Lb, gb = res["bf16"]
    for k in ("before", "after", "stop_token"):
        assert abs(Lb[k] - L[k]) < 1e-2 * abs(L[k]), (k, Lb[k], L[k])
    def cos(sel):
        u = np.concatenate([got[n].ravel() for n in sel])
        v = np.concatenate([gb[n].ravel() for n in sel])
        return float(u @ v / (np.linalg.norm(u) * np.linalg.norm(v)))
    ref = [n for n in fe if "/refnet/" in n]
    c_all, c_ref = cos(fe), cos(ref)
    print("adain bf16 vs fp32 gradient cosine: front end {:.5f}, refnet {:.5f}".format(c_all, c_ref))
    assert c_all > 0.97 and c_ref > 0.97


def test_train_config_adain_without_gpu():
    """train_config for args.adain: one 128-wide style embedding, no style classifiers / orthogonality
    loss (the AdaIN graph builds none, tacotron.py:485-495, 841)."""
    from tt2.train import train_config
    hp = small_hparams()
    cfg = train_config(hp, 4, 9, 6, frontend=True, n_emt=4, n_spk=2, style="adain")
    assert cfg.adain == 1 and cfg.use_gst == 0 and cfg.n_emt == 0 and cfg.n_spk == 0 and cfg.orthog_weight == 0
    assert cfg.memory_dim == 2 * hp.encoder_lstm_units + 128
    with pytest.raises(ValueError):
        train_config(hp, 4, 9, 6, frontend=False, style="adain")


def test_train_config_use_gst_without_gpu():
    """train_config carries hp.use_gst and the matching memory width (tacotron.py:284-291)."""
    from tt2.train import train_config
    hp = small_hparams()
    cfg = train_config(hp, 4, 9, 6, frontend=True)
    assert cfg.use_gst == 1 and cfg.memory_dim == 2 * hp.encoder_lstm_units + 2 * hp.style_embed_depth
    hp.override_from_dict(dict(use_gst=False))
    cfg = train_config(hp, 4, 9, 6, frontend=True)
    assert cfg.use_gst == 0 and cfg.memory_dim == 2 * hp.encoder_lstm_units + 256


@pytest.mark.gpu
def test_gpu_train_fused_encoder_lstm_matches_split_k_path():
    """The whole bf16 step from ids at the fork's encoder width (encoder_lstm_units 256): the
    encoder BiLSTM steps as fused products (k_tr_fused TF_EFWD / TF_EBWD: both directions' h·W_h +
    the cell in one launch per step, and dZ·W_h^T + the cell backward) against the split products
    + cell launches (TT2_TR_FUSED=0), like the decoder comparison: losses within 1e-5 relative, every
    gradient within 1e-2 (bf16 operand rounding level)."""
    import os
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(encoder_lstm_units=256, enc_conv_channels=128, embedding_dim=128))
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, B=6, T_in=23, T_out=8, T_ref=64)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    res = {}
    for mode in ("1", "0"):
        old = os.environ.get("TT2_TR_FUSED")
        os.environ["TT2_TR_FUSED"] = mode
        try:
            tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", frontend=True, max_T_ref=re.shape[1])
            try:
                tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
                L = tr.losses()
                g = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in TRN.frontend_var_names()}
            finally:
                tr.close()
        finally:
            if old is None:
                del os.environ["TT2_TR_FUSED"]
            else:
                os.environ["TT2_TR_FUSED"] = old
        res[mode] = (L, g)
    (La, ga), (Lb, gb) = res["1"], res["0"]
    for k in ("before", "after"):
        assert abs(La[k] - Lb[k]) < 1e-4 * abs(Lb[k]), (k, La[k], Lb[k])
    for n in ga:
        rel = float(np.linalg.norm(ga[n] - gb[n]) / max(np.linalg.norm(gb[n]), 1e-30))
        print("  {:90s} rel {:.3e}".format(n, rel))
        assert rel < 2e-2, (n, rel)


@pytest.mark.gpu
def test_gpu_train_im2col_gathered_large_products_match_kernels():
    """The whole bf16 step from ids with the Postnet conv weight gradients on gemm_bf16_kc's
    gathered operand (gemm.h KcConvA: the conv1d im2colᵀ written straight into the kernel's bf16
    copy, no fp32 columns) and the LSTM weight gradients transposed by its conversion pass, against
    TT2_TRAIN_BLAS=0 (fp32 transposes / im2colᵀ + gemm_x3_kernel).  The 512-channel Postnet convs
    are 2·5·512·512·(8·960) >= 2e10 flops, so the gathered form runs.  Losses within 1e-5 relative,
    every gradient within 2e-2 (bf16 operand rounding, K split / accumulation order)."""
    import os
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(reference_filters=[32, 32, 64, 64, 128, 128], postnet_channels=512))
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, B=8, T_in=11, T_out=960, T_ref=400)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    names = TRN.frontend_var_names() + TRN.postnet_var_names()
    res = {}
    old = os.environ.get("TT2_TRAIN_BLAS")
    try:
        for flag in ("1", "0"):
            os.environ["TT2_TRAIN_BLAS"] = flag
            tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", frontend=True, max_T_ref=re.shape[1])
            try:
                tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
                L = tr.losses()
                g = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
            finally:
                tr.close()
            res[flag] = (L, g)
    finally:
        if old is None:
            os.environ.pop("TT2_TRAIN_BLAS", None)
        else:
            os.environ["TT2_TRAIN_BLAS"] = old
    (La, ga), (Lb, gb) = res["1"], res["0"]
    for k in ("before", "after"):
        assert abs(La[k] - Lb[k]) < 1e-5 * abs(Lb[k]), (k, La[k], Lb[k])
    for n in ga:
        rel = float(np.linalg.norm(ga[n] - gb[n]) / max(np.linalg.norm(gb[n]), 1e-30))
        assert rel < 2e-2, (n, rel)


@pytest.mark.gpu
@pytest.mark.parametrize("T_out", [37, 300])
def test_gpu_train_postnet_planes_match_im2col(T_out):
    """bf16 training Postnet with the forward and input-gradient convolutions over padded bf16 planes
    (gemm.h conv_bf16_planes; the planes written by the BN forward / BN backward kernels) against
    the implicit-im2col gemm_x3_kernel convs (TT2_PN_PLANES=0), at 512 channels: after loss within
    1e-4 relative (measured 1.7e-5: a 3e-7 tanh difference flips the bf16 rounding of some next-layer
    inputs), every decoder and Postnet gradient within 2e-2 (bf16 operand rounding, tanh on
    v_exp/v_rcp against libm, accumulation order)."""
    import os
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(postnet_channels=512))
    B, T_in = 6, 17
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=3)
    names = TRN.train_var_names() + TRN.postnet_var_names()
    res = {}
    old = os.environ.get("TT2_PN_PLANES")
    try:
        for flag in ("1", "0"):
            os.environ["TT2_PN_PLANES"] = flag
            tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", postnet=True)
            try:
                tr.forward_backward(mem, lens, tg, st, pm, zm, pnm)
                L = tr.losses()
                g = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
            finally:
                tr.close()
            res[flag] = (L, g)
    finally:
        if old is None:
            os.environ.pop("TT2_PN_PLANES", None)
        else:
            os.environ["TT2_PN_PLANES"] = old
    (La, ga), (Lb, gb) = res["1"], res["0"]
    assert abs(La["after"] - Lb["after"]) < 1e-4 * abs(Lb["after"]), (La["after"], Lb["after"])
    for n in ga:
        den = np.linalg.norm(gb[n])
        if n.endswith("conv_layer_5_postnet_convolutions/conv1d/bias"):
            # conv -> training BN with no activation between: d bias = Σ dz = 0 up to rounding noise
            den = max(den, np.linalg.norm(gb[n.replace("/bias", "/kernel")]))
        rel = float(np.linalg.norm(ga[n] - gb[n]) / max(den, 1e-30))
        # the prenet's gradients move 2-6 % under any bf16 perturbation (bf16-rounded
        # pre-activations near zero flip ReLU decisions)
        assert rel < (6e-2 if "decoder_prenet" in n else 2e-2), (n, rel)


@pytest.mark.gpu
def test_gpu_train_encoder_planes_match_im2col():
    """bf16 step from ids with the text encoder's conv forward / input-gradient products over padded
    bf16 planes (conv_bf16_planes; the embedding's planes from k_rows_to_planes, the layers' from
    the BN forward / backward kernels) and the Postnet's, against TT2_PN_PLANES=0: losses within
    1e-4 relative, gradients within 5e-2 (measured up to 2.2e-2: the same bf16 operands summed in
    another order move the ReLU / BN-sensitive front-end gradients, e.g. the GST weight norm g, by
    about that much)."""
    import os
    from tt2.train import TacotronTrainer
    hp = small_hparams()
    hp.override_from_dict(dict(enc_conv_channels=128, embedding_dim=128, encoder_lstm_units=64))
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, B=6, T_in=23, T_out=8, T_ref=64)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    names = TRN.frontend_var_names() + TRN.postnet_var_names()
    res = {}
    old = os.environ.get("TT2_PN_PLANES")
    try:
        for flag in ("1", "0"):
            os.environ["TT2_PN_PLANES"] = flag
            tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", frontend=True, max_T_ref=re.shape[1])
            try:
                tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
                L = tr.losses()
                g = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}
            finally:
                tr.close()
            res[flag] = (L, g)
    finally:
        if old is None:
            os.environ.pop("TT2_PN_PLANES", None)
        else:
            os.environ["TT2_PN_PLANES"] = old
    (La, ga), (Lb, gb) = res["1"], res["0"]
    for k in ("before", "after"):
        assert abs(La[k] - Lb[k]) < 1e-4 * abs(Lb[k]), (k, La[k], Lb[k])
    for n in ga:
        den = np.linalg.norm(gb[n])
        if n.endswith("conv_layer_5_postnet_convolutions/conv1d/bias") or n.endswith("conv2d/bias"):
            # conv -> training BN with no activation between (Postnet layer 5, every refnet conv2d):
            # d bias = Σ dz = 0 up to rounding noise; measured against the kernel gradient's norm
            den = max(den, np.linalg.norm(gb[n.replace("/bias", "/kernel")]))
        rel = float(np.linalg.norm(ga[n] - gb[n]) / max(den, 1e-30))
        assert rel < 5e-2, (n, rel)


def _trainer_run(hp, W, case, env, postnet=False):
    """One bf16 forward/backward under the given TT2_* environment (read at context creation)."""
    import os
    from tt2.train import TacotronTrainer
    mem, lens, tg, st, pm, zm = case
    B, T_in, T_out = tg.shape[0], mem.shape[1], tg.shape[1]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", postnet=postnet)
        try:
            tr.forward_backward(mem, lens, tg, st, pm, zm)
            L = tr.losses()
            fr, sl, al = tr.outputs(T_in, T_out)
            g = {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in TRN.train_var_names()}
            gmem = tr.get("memory", 1, mem.shape)
            persist = float(tr.get("diag:persist", 0, (1,))[0])
            persist_bwd = float(tr.get("diag:persist_bwd", 0, (1,))[0])
        finally:
            tr.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return dict(L=L, fr=fr, sl=sl, al=al, g=g, gmem=gmem, persist=persist, persist_bwd=persist_bwd)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T_in,T_out,zmask", [(16, 40, 24, True), (5, 7, 3, False), (64, 150, 12, True)])
def test_gpu_train_persistent_forward_matches_launch_loop(B, T_in, T_out, zmask):
    """The persistent teacher-forced forward (train_persist.hip: one launch for the whole decoder
    loop, LSTM weights resident) against the per-step launch loop (TT2_TR_PERSIST=0) at the fork
    widths, bf16 step, ragged lengths: same operand rounding, different fp32 summation order
    (K split over waves, energies summed over attention-dim quarters).  Frames / stop logits within
    1e-3, alignments within 1e-4, losses within 1e-5 relative, every gradient within 1e-2
    (Frobenius, relative: the test_gpu_train_fused_lstm_matches_split_k_path tolerance)."""
    from tt2.hparams import hparams
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    assert memory_width(hp) == 1024
    W = init_tacotron_weights(hp, seed=5339)
    mem, lens, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=7)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=7)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=7) if zmask else None
    case = (mem, lens, tg, st, pm, zm)
    p = _trainer_run(hp, W, case, {"TT2_TR_PERSIST": "1"})
    q = _trainer_run(hp, W, case, {"TT2_TR_PERSIST": "0"})
    assert p["persist"] == 1.0 and q["persist"] == 0.0
    print("frames {:.3e} stop {:.3e} align {:.3e}".format(float(np.abs(p["fr"] - q["fr"]).max()),
                                                         float(np.abs(p["sl"] - q["sl"]).max()),
                                                         float(np.abs(p["al"] - q["al"]).max())))
    assert np.abs(p["fr"] - q["fr"]).max() < 1e-3
    assert np.abs(p["sl"] - q["sl"]).max() < 1e-3
    assert np.abs(p["al"] - q["al"]).max() < 1e-4
    for k in ("before", "stop_token"):
        assert abs(p["L"][k] - q["L"][k]) < 1e-5 * abs(q["L"][k]), (k, p["L"][k], q["L"][k])
    for n in list(p["g"]) + ["memory"]:
        a, b = (p["gmem"], q["gmem"]) if n == "memory" else (p["g"][n], q["g"][n])
        rel = float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
        print("  {:90s} rel {:.3e}".format(n, rel))
        assert rel < 1e-2, (n, rel)


@pytest.mark.gpu
def test_gpu_train_persistent_forward_close_to_oracle():
    """The persistent forward's bf16 step at the fork widths (D_mem 1024) against the float64
    oracle: the mixed-precision tolerance of test_gpu_train_bf16_gemms_close_to_oracle."""
    from tt2.hparams import hparams
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    B, T_in, T_out = 4, 37, 10
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    assert mem.shape[2] == 1024
    r = _trainer_run(hp, W, (mem, lens, tg, st, pm, zm), {"TT2_TR_PERSIST": "1"})
    assert r["persist"] == 1.0
    out, (b, s, _), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp))
    assert np.abs(r["fr"] - out["frames"]).max() < 1e-2
    assert np.abs(r["al"] - out["alignments"]).max() < 1e-3
    assert abs(r["L"]["before"] - b) < 1e-3 * b
    for n in TRN.train_var_names():
        frob = float(np.linalg.norm(r["g"][n] - g[n]) / max(np.linalg.norm(g[n]), 1e-30))
        print("  {:90s} frob {:.3e}".format(n, frob))
        assert frob < (0.1 if "prenet" in n else 1e-2), (n, frob)


@pytest.mark.gpu
def test_gpu_train_failed_persistent_forward_skips_update():
    """a persistent forward whose hand-off timed out (forced with the TT2_TP_FORCE_FAIL
    test hook, which writes the control word a stalled launch leaves) must not reach the weights.
    The step's status word behind the gradients (k_tr_status) makes clipped Adam and the BN moving
    averages skip the update -- on every rank, since the word rides in the tower mean -- and the
    read-back after the step reports the failure; the next good step updates normally."""
    import os
    from tt2._lib import TT2Error
    from tt2.hparams import hparams
    from tt2.train import TacotronTrainer
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    B, T_in, T_out = 5, 7, 3
    W = init_tacotron_weights(hp, seed=5339)
    mem, lens, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=7)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=7)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=7)
    name = TRN.L1 + "kernel"
    shape = np.asarray(W[name]).shape
    mm = "Tacotron_model/inference/postnet_convolutions/conv_layer_1_postnet_convolutions/batch_normalization/moving_mean"
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, precision="bf16", postnet=True)
    try:
        w0, m0 = tr.get(name, 0, shape), tr.get(mm, 0, (hp.postnet_channels,))
        os.environ["TT2_TP_FORCE_FAIL"] = "1"
        try:
            tr.forward_backward(mem, lens, tg, st, pm, None, pnm)
            tr.apply(1)
        finally:
            os.environ.pop("TT2_TP_FORCE_FAIL", None)
        with pytest.raises(TT2Error, match="timed out"):
            tr.losses()
        assert float(tr.get("diag:persist", 0, (1,))[0]) == 1.0
        assert float(tr.grad_buf[-1].item()) == 1.0          # the status word
        np.testing.assert_array_equal(tr.get(name, 0, shape), w0)
        np.testing.assert_array_equal(tr.get(mm, 0, (hp.postnet_channels,)), m0)
        np.testing.assert_array_equal(tr.get(name, 2, shape), 0.0)   # Adam m untouched
        tr.forward_backward(mem, lens, tg, st, pm, None, pnm)
        tr.apply(1)
        L = tr.losses()
        assert np.isfinite(L["loss"]) and float(tr.grad_buf[-1].item()) == 0.0
        assert np.abs(tr.get(name, 0, shape) - w0).max() > 0
    finally:
        tr.close()


_LOSS_KEYS = ("before", "after", "stop_token", "regularization", "style_emb_loss_emt", "style_emb_loss_spk",
              "style_emb_orthog_loss")


def _configs4_case(T_out, T_ref=800, B=64, T_in=150):
    """The bench's configs[4] batch (bench.py bench_train: seeds, 4 + 4 style classes, synthetic
    labels) at a chosen T_out."""
    from tt2.hparams import hparams
    from tt2.synthetic import enc_conv_masks, enc_zoneout_masks, tacotron_inputs
    from tt2.train import init_style_disc_weights
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    W = init_tacotron_weights(hp, seed=hp.tacotron_random_seed)
    W.update(init_style_disc_weights(hp, 4, 4))
    _, _, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=1234)
    ids, tl, re, rs = tacotron_inputs(B, T_in, T_ref, seed=1234)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=7)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=7)
    pnm = postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=7)
    em = enc_conv_masks(hp.enc_conv_num_layers, B, T_in, hp.enc_conv_channels, seed=7)
    ezm = enc_zoneout_masks(T_in, B, hp.encoder_lstm_units, seed=7)
    lab = np.random.default_rng(99).integers(0, 4, (2, B)).astype(np.int32)
    return hp, W, (ids, tl, re, rs, tg, st, pm, zm, pnm, em, ezm), lab


@pytest.mark.gpu
def test_gpu_train_configs4_whole_step_fp32_bf16_agree():
    """the whole configs[4] step at full size (B = 64, T_in = 150, T_ref = 800,
    T_out = 800, from ids with the front end, 4 + 4 class style classifiers and the orthogonality
    loss): fp32 and bf16 agree on every loss component -- the decoder / Postnet losses within 1e-3,
    the style losses within 5e-3 (both reference encoders' conv and GRU products take bf16 operands,
    2^-9 relative rounding, and the orthogonality loss multiplies two of their outputs) -- and on the
    global gradient norm within 2 %; everything finite."""
    from tt2.train import TacotronTrainer
    hp, W, batch, lab = _configs4_case(800)
    res = {}
    for prec in ("fp32", "bf16"):
        tr = TacotronTrainer(hp, W, 64, 150, 800, 0, precision=prec, frontend=True, max_T_ref=800, n_emt=4, n_spk=4)
        try:
            tr.set_style_labels(lab[0], lab[1])
            tr.forward_backward_text(*batch)
            tr.apply(1)
            res[prec] = tr.losses()
        finally:
            tr.close()
        print(prec, {k: round(v, 5) for k, v in res[prec].items()})
        assert all(np.isfinite(v) for v in res[prec].values())
    for k in _LOSS_KEYS:
        a, b = res["fp32"][k], res["bf16"][k]
        tol = 5e-3 if k.startswith("style") else 1e-3
        assert abs(a - b) <= tol * abs(a), (k, a, b)
    a, b = res["fp32"]["grad_norm"], res["bf16"]["grad_norm"]
    assert abs(a - b) < 2e-2 * a, (a, b)


@pytest.mark.gpu
def test_gpu_train_configs4_trajectory_matches_oracle():
    """the whole configs[4] step at its full widths and shapes -- B = 64 (two
    32-row blocks), T_in = 150, both reference encoders over T_ref = 800 (6 stride-2 convs with
    batch-statistics BN, the GRU), 4 + 4 class style classifiers, orthogonality loss, Postnet --
    with T_out reduced to 6 so the float64 oracle (oracle/train_ref.py) runs in seconds: the fp32
    device's per-component losses over three clipped-Adam updates at lr 1e-3 follow the oracle's
    (losses before update 1 within 1e-4 relative, before updates 2 and 3 within 2e-3; the global
    gradient norm of each update within 1e-3).  This is the trajectory the bench reports at T_out =
    800 (the orthogonality loss jumps after the first sign-sized Adam step)."""
    from tt2.train import TacotronTrainer
    T = 6
    hp, W, batch, lab = _configs4_case(T)
    ids, tl, re, rs, tg, st, pm, zm, pnm, em, ezm = batch
    style = dict(emt_labels=lab[0], spk_labels=lab[1], n_emt=4, n_spk=4, orthog_weight=0.02)
    names = (TRN.frontend_var_names() + TRN.style_disc_var_names(False, 4, 4) + TRN.train_var_names()
             + TRN.postnet_var_names())
    tr = TacotronTrainer(hp, W, 64, 150, T, 0, precision="fp32", frontend=True, max_T_ref=800, n_emt=4, n_spk=4)
    dev = []
    try:
        tr.set_style_labels(lab[0], lab[1])
        for step in (1, 2, 3):
            tr.forward_backward_text(*batch)
            tr.apply(step, lr=1e-3)
            dev.append(tr.losses())
    finally:
        tr.close()
    params = {n: np.asarray(W[n], np.float64) for n in names}
    m = {n: np.zeros_like(p) for n, p in params.items()}
    v = {n: np.zeros_like(p) for n, p in params.items()}
    for step in (1, 2, 3):
        Wc = dict(W)
        Wc.update(params)
        L, g, _ = TRN.train_grads_frontend(Wc, ids, tl, re, rs, tg, st, pm, zm, em, ezm, hp.tacotron_reg_weight,
                                           postnet_masks=pnm, style=style)
        ref = dict(zip(("before", "stop_token", "regularization", "after", "style_emb_loss_emt",
                        "style_emb_loss_spk", "style_emb_orthog_loss"), L))
        gn = TRN.clip_and_adam(params, {n: g[n] for n in names}, m, v, step, 1e-3, eps=hp.tacotron_adam_epsilon)
        got = dev[step - 1]
        print(step, {k: (round(got[k], 5), round(ref[k], 5)) for k in ref}, "gnorm", got["grad_norm"], gn)
        tol = 1e-4 if step == 1 else 2e-3
        for k, want in ref.items():
            assert abs(got[k] - want) <= tol * abs(want) + 1e-7, (step, k, got[k], want)
        assert abs(got["grad_norm"] - gn) < 1e-3 * gn, (step, got["grad_norm"], gn)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T_in,T_out,zmask", [(5, 7, 3, False), (16, 40, 24, True), (64, 150, 12, True),
                                                 (64, 160, 6, True), (33, 129, 17, False), (8, 192, 4, True)])
def test_gpu_train_persistent_backward_matches_launch_loop(B, T_in, T_out, zmask):
    """The persistent BPTT backward (train_bwd_persist.hip: one launch for the whole reverse decoder loop,
    LSTM weight blocks and the values quarter resident) against the per-step backward launches
    (TT2_TR_PERSIST_BWD=0), both after the persistent forward, fork widths, bf16 step, ragged lengths:
    the same bf16 operand rounding, different fp32 summation orders (K-block partials, the d align
    quarters, the location-conv backward folded through KW).  Every gradient within 1e-2 (Frobenius,
    relative: the tolerance of the fused and persistent-forward A/B tests), losses identical."""
    from tt2.hparams import hparams
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    W = init_tacotron_weights(hp, seed=5339)
    mem, lens, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=7)
    pm = prenet_masks(T_out, B, hp.prenet_layers[0], seed=7)
    zm = zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=7) if zmask else None
    case = (mem, lens, tg, st, pm, zm)
    p = _trainer_run(hp, W, case, {"TT2_TR_PERSIST_BWD": "1"})
    q = _trainer_run(hp, W, case, {"TT2_TR_PERSIST_BWD": "0"})
    assert p["persist"] == 1.0 and q["persist"] == 1.0
    # T_in beyond the backward's 160-position capacity (train_bwd_persist.h TB_TMAX) runs the launches
    assert p["persist_bwd"] == (1.0 if T_in <= 160 else 0.0) and q["persist_bwd"] == 0.0
    for k in ("before", "stop_token"):
        assert p["L"][k] == q["L"][k], (k, p["L"][k], q["L"][k])
    for n in list(p["g"]) + ["memory"]:
        a, b = (p["gmem"], q["gmem"]) if n == "memory" else (p["g"][n], q["g"][n])
        rel = float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
        print("  {:90s} rel {:.3e}".format(n, rel))
        assert np.isfinite(a).all()
        assert rel < 1e-2, (n, rel)


@pytest.mark.gpu
def test_gpu_train_persistent_backward_close_to_oracle():
    """The persistent backward's bf16 step at the fork widths against the float64 oracle: the
    mixed-precision tolerance of test_gpu_train_persistent_forward_close_to_oracle."""
    from tt2.hparams import hparams
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    B, T_in, T_out = 4, 37, 10
    W, mem, lens, tg, st, pm, zm = _case(hp, B, T_in, T_out)
    r = _trainer_run(hp, W, (mem, lens, tg, st, pm, zm), {"TT2_TR_PERSIST": "1", "TT2_TR_PERSIST_BWD": "1"})
    assert r["persist"] == 1.0 and r["persist_bwd"] == 1.0
    out, (b, s, _), g = TRN.train_grads(W, mem, lens, tg, st, pm, zm, hp.tacotron_reg_weight, clip=_clip(hp))
    assert abs(r["L"]["before"] - b) < 1e-3 * b
    for n in TRN.train_var_names() + ["memory"]:
        got, want = (r["gmem"], g["memory"]) if n == "memory" else (r["g"][n], g[n])
        frob = float(np.linalg.norm(got - want) / max(np.linalg.norm(want), 1e-30))
        print("  {:90s} frob {:.3e}".format(n, frob))
        assert frob < (0.1 if "prenet" in n else 1e-2), (n, frob)


@pytest.mark.gpu
@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 2e-2)])
def test_gpu_refnet_conv_backward_direct_matches_im2col(precision, tol):
    """The refnet conv2d backward without a materialised im2col (k_fe_conv2d_dw: LDS-staged patches,
    fp32 FMA, partial rows summed; k_fe_conv2d_dx: the input gradient as a gather over the taps)
    against the im2colᵀ + GEMM + col2im form (TT2_FE_CONV_DIRECT=0) at the fork widths (filters
    32, 32, 64, 64, 128, 128: the direct kernels take layers 0-3 / 1-2, the rest stay on the GEMM
    form) with T_ref = 96 (odd pads on the way down), and the first layer's forward conv
    (k_fe_conv2d_fwd_small) against the implicit GEMM.  fp32: both forms are fp32-grade (the
    forward's fp32 FMA against split fp16x3 moves every later gradient by ~2e-5): every gradient
    within 1e-4 of its max; bf16: the moved forward re-rounds the whole bf16 step, so losses within
    1e-5 and the global gradient norm within 2 % (the criteria of the configs[4] fp32-vs-bf16 test)."""
    import os
    from tt2.hparams import hparams
    from tt2.train import TacotronTrainer
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, B=4, T_in=12, T_out=6, T_ref=96)
    names = TRN.frontend_var_names() + TRN.train_var_names() + TRN.postnet_var_names()
    out = []
    for direct in ("1", "0"):
        old = os.environ.get("TT2_FE_CONV_DIRECT")
        os.environ["TT2_FE_CONV_DIRECT"] = direct
        try:
            tr = TacotronTrainer(hp, W, 4, 12, 6, 0, frontend=True, max_T_ref=96, precision=precision)
        finally:
            if old is None:
                os.environ.pop("TT2_FE_CONV_DIRECT", None)
            else:
                os.environ["TT2_FE_CONV_DIRECT"] = old
        try:
            tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
            L = tr.losses()
            out.append((L, {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}))
        finally:
            tr.close()
    (La, ga), (Lb, gb) = out
    assert abs(La["loss"] - Lb["loss"]) < 1e-5 * abs(Lb["loss"])
    if precision == "bf16":
        na = np.sqrt(sum(float((ga[n].astype(np.float64) ** 2).sum()) for n in names))
        nb = np.sqrt(sum(float((gb[n].astype(np.float64) ** 2).sum()) for n in names))
        assert abs(na - nb) < tol * nb, (na, nb)
        return
    # (a conv bias ahead of batch norm has a zero gradient: rounding noise of ~1e-9 both ways)
    live = [n for n in names if np.abs(gb[n]).max() > 1e-6]
    worst = max(live, key=lambda n: _rel(ga[n], gb[n]))
    for n in names:
        if "refnet" in n and "conv2d/kernel" in n:
            assert n in live, n
        if n in live:
            assert _rel(ga[n], gb[n]) < tol, (n, _rel(ga[n], gb[n]), worst)
        else:
            assert np.abs(ga[n]).max() < 1e-6, n


@pytest.mark.gpu
@pytest.mark.parametrize("precision,tol,ltol", [("fp32", 1e-4, 1e-5), ("bf16", 2e-2, 1e-3)])
def test_gpu_refnet_gru_sequence_kernels_match_per_step(precision, tol, ltol):
    """The refnet GRU recurrence in one work-group per direction (k_fe_gru_fwd_seq / k_fe_gru_bwd_seq:
    recurrent weights register-resident as fp32 MFMA fragments) against the per-step launches
    (TT2_FE_GRU_SEQ=0: the two recurrent products per step on the GEMM kernels + the cell kernels) at
    the fork widths (reference_depth 128, T_ref = 400: 7 GRU steps): every gradient
    of the step relative to its max and the losses.  fp32: both fp32-grade (1e-4 after the
    recurrence; losses 1e-5); bf16: the per-step products round to bf16, the sequence kernels stay
    fp32, and the moved style embedding re-rounds the whole bf16 step (losses 1e-3, global gradient
    norm 2 %, the criteria of the configs[4] fp32-vs-bf16 test)."""
    import os
    from tt2.hparams import hparams
    from tt2.train import TacotronTrainer
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, B=4, T_in=12, T_out=6, T_ref=400)
    names = TRN.frontend_var_names() + TRN.train_var_names() + TRN.postnet_var_names()
    out = []
    for seq in ("1", "0"):
        old = os.environ.get("TT2_FE_GRU_SEQ")
        os.environ["TT2_FE_GRU_SEQ"] = seq
        try:
            tr = TacotronTrainer(hp, W, 4, 12, 6, 0, frontend=True, max_T_ref=400, precision=precision)
        finally:
            if old is None:
                os.environ.pop("TT2_FE_GRU_SEQ", None)
            else:
                os.environ["TT2_FE_GRU_SEQ"] = old
        try:
            tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
            L = tr.losses()
            out.append((L, {n: tr.get(n, 1, np.asarray(W[n]).shape) for n in names}))
        finally:
            tr.close()
    (La, ga), (Lb, gb) = out
    assert abs(La["loss"] - Lb["loss"]) < ltol * abs(Lb["loss"])
    if precision == "bf16":  # the moved style embedding re-rounds the whole bf16 step: global norm only
        na = np.sqrt(sum(float((ga[n].astype(np.float64) ** 2).sum()) for n in names))
        nb = np.sqrt(sum(float((gb[n].astype(np.float64) ** 2).sum()) for n in names))
        assert abs(na - nb) < tol * nb, (na, nb)
        return
    live = [n for n in names if np.abs(gb[n]).max() > 1e-6]
    worst = max(live, key=lambda n: _rel(ga[n], gb[n]))
    for n in names:
        if "gru_cell" in n:
            assert n in live, n
        if n in live:
            assert _rel(ga[n], gb[n]) < tol, (n, _rel(ga[n], gb[n]), worst)
        else:
            assert np.abs(ga[n]).max() < 1e-6, n
