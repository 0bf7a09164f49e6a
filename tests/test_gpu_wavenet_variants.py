"""GPU parity of the WaveNet front/back-end variants: every upsample_type
of wavenet.py:163-203 (2D / 1D / Resize / SubPixel / NearestNeighbor, ReLU / LeakyReLU / no
activation, SubPixel with NN_init off) and the Gaussian output head (gaussian.py:39-52), against
oracle/wavenet_ref.py.  Upsampled conditioning within 1e-5; Gaussian samples within 1e-5 given the
same injected N(0,1) draws (no argmax: the Gaussian head has no discrete choice)."""
import numpy as np
import pytest

from _common import mol_uniforms, small_wavenet_hparams, wavenet_oracle_hp
from oracle import wavenet_ref as WR

pytestmark = pytest.mark.gpu


def _hp(**kw):
    hp = small_wavenet_hparams(6, 2)
    hp.override_from_dict(kw)
    return hp


@pytest.mark.parametrize("ut,act,scales,nn_init", [
    ("2D", "LeakyRelu", [5, 5, 11], True),
    ("2D", None, [5, 5, 11], True),
    ("1D", "Relu", [5, 5, 11], True),
    ("Resize", "Relu", [5, 5, 11], True),
    ("Resize", "LeakyRelu", [11, 25], True),
    ("SubPixel", "Relu", [11, 25], True),
    ("SubPixel", "LeakyRelu", [5, 5, 11], False),
    ("NearestNeighbor", "Relu", [5, 5, 11], True),
])
def test_upsample_network(ut, act, scales, nn_init):
    from tt2.engine import WaveNetEngine
    from tt2.weights import init_wavenet_weights
    hop = int(np.prod(scales))
    hp = _hp(upsample_type=ut, upsample_activation=act, upsample_scales=scales, hop_size=hop,
             NN_init=nn_init)
    W = init_wavenet_weights(hp, seed=77)
    rng = np.random.default_rng(len(ut) + len(scales))
    B, T_f = 2, 3
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32))
    T = T_f * hop
    um, ul = mol_uniforms(T, B, seed=5)
    eng = WaveNetEngine(hp, W, B, T, 0)
    out = eng.generate(cond, um, ul, 0, None, want_upsampled=True)
    eng.close()
    ref = WR.upsample_network(cond.transpose(0, 2, 1), W, wavenet_oracle_hp(hp))
    assert out["upsampled"].shape == ref.shape == (B, 80, T)
    np.testing.assert_allclose(out["upsampled"], ref, rtol=0, atol=1e-5)


@pytest.mark.parametrize("teacher", [True, False])
def test_gaussian_head(teacher):
    from tt2.engine import WaveNetEngine
    from tt2.weights import init_wavenet_weights
    hp = _hp(out_channels=2)
    W = init_wavenet_weights(hp, seed=31)
    rng = np.random.default_rng(4)
    B, T_f = 2, 1
    T = T_f * 275
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32))
    normals = rng.standard_normal((T, B)).astype(np.float32) * np.float32(0.3)
    tg = rng.uniform(-0.9, 0.9, (B, T)).astype(np.float32) if teacher else None
    eng = WaveNetEngine(hp, W, B, T, 0)
    out = eng.generate(cond, None, normals, 0, tg, want_logits=True, want_upsampled=True)
    eng.close()
    c_up = WR.upsample_network(cond.transpose(0, 2, 1), W, wavenet_oracle_hp(hp))
    y, k, lg = WR.incremental(c_up.transpose(0, 2, 1), W, wavenet_oracle_hp(hp), None, normals, tg,
                              return_logits=True)
    assert out["logits"].shape == (B, T, 2)
    np.testing.assert_array_equal(out["k"], 0)
    # teacher-forced: every step independent; free-running: the chain stays within 1e-4
    np.testing.assert_allclose(out["logits"], lg, atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(out["y"], y, atol=1e-4)


def test_gaussian_device_rng_is_standard_normal():
    """Gaussian head with the on-device Box-Muller draws: with the last 1x1 zeroed and bias
    [0, log 0.1] every sample is clip(0.1 · n) = 0.1 · n, so n must look standard normal."""
    from tt2.engine import WaveNetEngine
    from tt2.weights import init_wavenet_weights
    hp = _hp(out_channels=2)
    W = init_wavenet_weights(hp, seed=32)
    pre = "WaveNet_model/inference/skip_convolutions/final_convolution_2/"
    W[pre + "kernel"] = np.zeros_like(W[pre + "kernel"])
    W[pre + "bias"] = np.array([0.0, np.log(0.1)], np.float32)
    rng = np.random.default_rng(6)
    T = 16 * 275
    cond = WR.interp_condition(rng.uniform(-4, 4, (1, 16, 80)).astype(np.float32))
    eng = WaveNetEngine(hp, W, 1, T, 0)
    out = eng.generate(cond, None, None, 123, None)
    eng.close()
    n = out["y"][0].astype(np.float64) / 0.1
    assert abs(n.mean()) < 0.1 and 0.9 < n.var() < 1.1
    assert abs(np.mean(n ** 3)) < 0.25 and 2.5 < np.mean(n ** 4) < 3.5   # symmetric, Gaussian tails
    assert len(np.unique(out["y"][0])) > T - 5                          # a fresh draw per sample


@pytest.mark.parametrize("R,mode", [(64, "ids"), (64, "features"), (128, "ids"), (256, "features")])
def test_global_conditioning(R, mode):
    """Global conditioning (wavenet.py:152-158, 770-775; modules.py:427-433, 505-509): speaker ids
    through the gc_embedding table, or the g features themselves; every layer's conv1x1g term joins
    both gate halves.  Teacher-forced logits within 1e-4 of the oracle at the narrow pipe (R = 64)
    and the wide generator (R = 128 one-hop, R = 256 two-hop), rows of different speakers differ,
    and the Synthesizer shim passes speaker ids through.  A batch other than the one the global
    condition was set for is refused (stale rows would be used otherwise)."""
    from tt2.engine import WaveNetEngine
    from tt2.weights import init_wavenet_weights
    kw = dict(gin_channels=16, use_speaker_embedding=(mode == "ids"), n_speakers=5)
    if R != 64:
        kw.update(residual_channels=R, gate_channels=2 * R, skip_out_channels=R)
    hp = _hp(**kw)
    W = init_wavenet_weights(hp, seed=41)
    rng = np.random.default_rng(9)
    B, T_f = 2, 1
    T = T_f * 275
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32))
    um, ul = mol_uniforms(T, B, seed=6)
    tg = rng.uniform(-0.9, 0.9, (B, T)).astype(np.float32)
    g = np.array([3, 1], np.int32) if mode == "ids" else rng.normal(0, 0.5, (B, 16)).astype(np.float32)
    eng = WaveNetEngine(hp, W, B, T, 0)
    with pytest.raises(ValueError):
        eng.generate(cond, um, ul, 0, tg)                      # gin_channels > 0 needs g
    out = eng.generate(cond, um, ul, 0, tg, want_logits=True, g=g)
    same = eng.generate(np.repeat(cond[:1], 2, 0), um, ul, 0, np.repeat(tg[:1], 2, 0), want_logits=True, g=g)
    eng.close()
    ohp = wavenet_oracle_hp(hp)
    c_up = WR.upsample_network(cond.transpose(0, 2, 1), W, ohp)
    _, _, lg = WR.incremental(c_up.transpose(0, 2, 1), W, ohp, um, ul, tg, return_logits=True, g=g)
    np.testing.assert_allclose(out["logits"], lg, atol=1e-4, rtol=1e-4)
    from tt2._lib import TT2Error, ptr
    eng1 = WaveNetEngine(hp, W, B, T, 0)
    eng1.set_global_condition(g, B)                        # set for B rows, generate 1: refused
    c1 = np.ascontiguousarray(cond[:1])
    y1 = np.zeros((1, T), np.float32)
    with pytest.raises(TT2Error, match="exactly these B rows"):
        eng1._ok(eng1.lib.tt2_wn_generate(eng1.h, ptr(c1), 1, T_f, ptr(np.ascontiguousarray(um[:, :1])),
                                          ptr(np.ascontiguousarray(ul[:, :1])), 0, None, ptr(y1), None, None,
                                          None))
    eng1.close()
    # identical conditioning and inputs, different global condition -> different logits
    assert np.abs(same["logits"][0] - same["logits"][1]).max() > 1e-3
    if mode == "ids":
        from wavenet_vocoder.synthesizer import Synthesizer
        syn = Synthesizer()
        syn.load(None, hp)
        syn.model.load_weights(W)
        mels = [rng.uniform(-4, 4, (1, 80)).astype(np.float32) for _ in range(B)]
        wavs = syn.synthesize(mels, [3, 1], None, None, None, u_mix=um, u_log=ul)
        assert len(wavs) == B and all(w.shape == (275,) for w in wavs)
