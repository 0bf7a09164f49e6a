"""WaveNet 'mulaw-quantize' input with the softmax head (wavenet.py:433-452: one-hot input of
quantize_channels classes, tf.multinomial over the logits, inv_mulaw_quantize of the draw) and
unconditional synthesis (cin_channels <= 0, wavenet.py:410-411), HIP path (k_generate_q and the
scalar-input generators with a zero condition) against the numpy oracle.  The sampler's uniforms
are injected (u_log [T, B]); TF's multinomial kernel is restated in oracle/wavenet_ref.py
(categorical_sample).  Tolerances: logits 1e-4; classes exact where the oracle's cdf margin to
u·total exceeds 1e-6 of the total (the two sides sum the float64 cdf in different orders)."""
import numpy as np
import pytest

from _common import mol_uniforms, small_wavenet_hparams, wavenet_oracle_hp
from oracle import wavenet_ref as WR

pytestmark = pytest.mark.gpu


def _quant_hp(layers=6, stacks=2, Q=256, cin=80):
    hp = small_wavenet_hparams(layers, stacks)
    hp.override_from_dict(dict(input_type="mulaw-quantize", quantize_channels=Q, out_channels=Q,
                               cin_channels=cin))
    return hp


def _margin_ok(lg, u, k_ref):
    """classes whose oracle draw is not within 1e-6·total of a cdf boundary"""
    lg = lg.astype(np.float64)
    e = np.exp(lg - lg.max(-1, keepdims=True))
    cdf = np.cumsum(e, -1)
    tot = cdf[..., -1]
    tgt = u * tot
    kk = k_ref.astype(np.int64)
    hi = np.take_along_axis(cdf, kk[..., None], -1)[..., 0]
    lo = np.where(kk > 0, np.take_along_axis(cdf, np.maximum(kk - 1, 0)[..., None], -1)[..., 0], 0.0)
    return np.minimum(hi - tgt, tgt - lo) > 1e-6 * tot


def _eng(hp, W, B, T):
    from tt2.engine import WaveNetEngine
    return WaveNetEngine(hp, W, B, T, 0)


@pytest.mark.parametrize("layers,stacks,B,T_f", [(6, 2, 2, 1), (24, 4, 1, 1)])
def test_quantize_teacher_forced_matches_oracle(layers, stacks, B, T_f):
    from tt2.weights import init_wavenet_weights
    hp = _quant_hp(layers, stacks)
    W = init_wavenet_weights(hp, seed=5339)
    assert W["WaveNet_model/inference/input_convolution/kernel"].shape == (1, 256, hp.residual_channels)
    rng = np.random.default_rng(31)
    T = T_f * 275
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32))
    _, ul = mol_uniforms(T, B, seed=4)
    teacher = rng.integers(0, 256, (B, T)).astype(np.float32)
    eng = _eng(hp, W, B, T)
    out = eng.generate(cond, None, ul, 0, teacher, want_logits=True)
    eng.close()
    c_up = WR.upsample_2d(cond.transpose(0, 2, 1), W, hp.upsample_scales)
    y, k, lg = WR.incremental(c_up.transpose(0, 2, 1), W, wavenet_oracle_hp(hp), None, ul, teacher,
                              return_logits=True)
    np.testing.assert_allclose(out["logits"], lg, atol=1e-4, rtol=1e-4)
    safe = _margin_ok(lg, ul.T, k)
    assert safe.mean() > 0.99
    np.testing.assert_array_equal(out["k"][safe], k[safe])
    np.testing.assert_allclose(out["y"], WR.inv_mulaw_quantize_f32(out["k"]), atol=1e-6)
    np.testing.assert_allclose(out["y"][safe], y[safe], atol=1e-6)


def test_quantize_free_run_prefix():
    from tt2.weights import init_wavenet_weights
    hp = _quant_hp(6, 2)
    W = init_wavenet_weights(hp, seed=77)
    rng = np.random.default_rng(12)
    B, T = 2, 275
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, 1, 80)).astype(np.float32))
    _, ul = mol_uniforms(T, B, seed=9)
    eng = _eng(hp, W, B, T)
    out = eng.generate(cond, None, ul, 0, None)
    eng.close()
    c_up = WR.upsample_2d(cond.transpose(0, 2, 1), W, hp.upsample_scales)
    y, k = WR.incremental(c_up.transpose(0, 2, 1), W, wavenet_oracle_hp(hp), None, ul)
    for b in range(B):
        same = out["k"][b] == k[b]
        first_diff = int(np.argmin(same)) if not same.all() else T
        assert first_diff >= 200
        np.testing.assert_allclose(out["y"][b, :first_diff], y[b, :first_diff], atol=1e-6)


@pytest.mark.parametrize("quant", [False, True])
def test_unconditional_matches_oracle(quant):
    """cin_channels = -1: no conv1x1c, no upsampler (wavenet.py:410-411); teacher-forced logits"""
    from tt2.weights import init_wavenet_weights
    hp = _quant_hp(6, 2, cin=-1) if quant else small_wavenet_hparams(6, 2)
    if not quant:
        hp.override_from_dict(dict(cin_channels=-1))
    W = init_wavenet_weights(hp, seed=5339)
    assert not any("cin_conv" in n or "upsampling" in n for n in W)
    rng = np.random.default_rng(41)
    B, T = 2, 300
    um, ul = mol_uniforms(T, B, seed=6)
    teacher = (rng.integers(0, 256, (B, T)) if quant else rng.uniform(-0.9, 0.9, (B, T))).astype(np.float32)
    eng = _eng(hp, W, B, T)
    out = eng.generate_unconditional(B, T, None if quant else um, ul, 0, teacher, want_logits=True)
    eng.close()
    y, k, lg = WR.incremental(None, W, wavenet_oracle_hp(hp), None if quant else um, ul, teacher,
                              return_logits=True, T=T)
    np.testing.assert_allclose(out["logits"], lg, atol=1e-4, rtol=1e-4)


def test_quantize_fork_widths_teacher_forced():
    """the fork's WaveNet widths (hparams.py:222-239: R = 128, 20 layers / 2 stacks) with the
    mulaw-quantize input and a 256-class softmax head"""
    import time
    from tt2.hparams import hparams
    from tt2.weights import init_wavenet_weights
    hp = hparams.copy()
    hp.override_from_dict(dict(input_type="mulaw-quantize", quantize_channels=256, out_channels=256,
                               wavenet_num_gpus=1, hop_size=275))  # [11, 25] upsampler (test_gpu_wavenet_wide)
    W = init_wavenet_weights(hp, seed=5339)
    rng = np.random.default_rng(8)
    B, T_f = 1, 2
    hop = int(np.prod(hp.upsample_scales))
    T = T_f * hop
    cond = WR.interp_condition(rng.uniform(-4, 4, (B, T_f, hp.num_mels)).astype(np.float32))
    _, ul = mol_uniforms(T, B, seed=2)
    teacher = rng.integers(0, 256, (B, T)).astype(np.float32)
    eng = _eng(hp, W, B, T)
    eng.generate(cond, None, ul, 0, teacher)
    t0 = time.perf_counter()
    out = eng.generate(cond, None, ul, 0, teacher, want_logits=True)
    dt = time.perf_counter() - t0
    eng.close()
    print("fork-width mulaw-quantize: {:.1f} us/sample".format(dt / T * 1e6))
    ohp = wavenet_oracle_hp(hp)
    c_up = WR.upsample_network(cond.transpose(0, 2, 1), W, ohp)
    y, k, lg = WR.incremental(c_up.transpose(0, 2, 1), W, ohp, None, ul, teacher, return_logits=True)
    np.testing.assert_allclose(out["logits"], lg, atol=1e-4, rtol=1e-4)
    safe = _margin_ok(lg, ul.T, k)
    np.testing.assert_array_equal(out["k"][safe], k[safe])


@pytest.mark.parametrize("quant", [False, True])
def test_synthesizer_unconditional_path(quant):
    """wavenet_vocoder.synthesizer.Synthesizer without local conditioning (synthesizer.py:51-53,
    75-78): synthesis_length = 100 samples per row, trimmed to len(mel) * hop like the reference's
    audio_lengths; the generated row equals the engine's own unconditional run on the same uniforms,
    and its logits (teacher-forced on the produced samples) match the oracle within 1e-4."""
    from wavenet_vocoder.synthesizer import SYNTHESIS_LENGTH, Synthesizer
    hp = _quant_hp(6, 2, cin=-1) if quant else small_wavenet_hparams(6, 2)
    if not quant:
        hp.override_from_dict(dict(cin_channels=-1))
    T = SYNTHESIS_LENGTH
    um, ul = mol_uniforms(T, 1, seed=13)
    syn = Synthesizer()
    syn.load(None, hp)
    wavs = syn.synthesize(None, None, None, None, None, u_mix=None if quant else um, u_log=ul)
    assert len(wavs) == 1 and wavs[0].shape == (T,)
    W = syn.model._weights
    eng = _eng(hp, W, 1, T)
    out = eng.generate_unconditional(1, T, None if quant else um, ul, 0, None)
    eng.close()
    np.testing.assert_array_equal(wavs[0], out["y"][0])
    # with mels given, the rows are trimmed to len(mel) * hop (here shorter than 100 samples)
    short = syn.synthesize([np.zeros((0, 80), np.float32)], None, None, None, None,
                           u_mix=None if quant else um, u_log=ul)
    assert short[0].shape == (0,)
    teacher = (out["k"] if quant else out["y"]).astype(np.float32)
    eng = _eng(hp, W, 1, T)
    tf = eng.generate_unconditional(1, T, None if quant else um, ul, 0, teacher, want_logits=True)
    eng.close()
    _, _, lg = WR.incremental(None, W, wavenet_oracle_hp(hp), None if quant else um, ul, teacher,
                              return_logits=True, T=T)
    np.testing.assert_allclose(tf["logits"], lg, atol=1e-4, rtol=1e-4)


def test_synthesizer_debug_wavs_teacher_force(tmp_path):
    """hparams.wavenet_synth_debug (synthesizer.py:56-58, 83-95): the mels come from
    wavenet_debug_mels and the debug wavs teacher-force the generator; the result equals the
    engine's teacher-forced generation on the same condition and uniforms."""
    from wavenet_vocoder.synthesizer import Synthesizer, _interp
    hp = small_wavenet_hparams(6, 2)
    rng = np.random.default_rng(5)
    hop = int(np.prod(hp.upsample_scales))
    mel = rng.uniform(-4, 4, (2, 80)).astype(np.float32)
    wav = rng.uniform(-0.5, 0.5, (2 * hop,)).astype(np.float32)
    np.save(tmp_path / "mel.npy", mel)
    np.save(tmp_path / "audio.npy", wav)
    hp.override_from_dict(dict(wavenet_synth_debug=True, wavenet_debug_mels=[str(tmp_path / "mel.npy")],
                               wavenet_debug_wavs=[str(tmp_path / "audio.npy")]))
    um, ul = mol_uniforms(2 * hop, 1, seed=3)
    syn = Synthesizer()
    syn.load(None, hp)
    got = syn.synthesize([np.zeros((7, 80), np.float32)], None, None, None, None, u_mix=um, u_log=ul)
    assert len(got) == 1 and got[0].shape == (2 * hop,)
    cond = _interp(np.clip(mel, -4, 4), (-4, 4))[None].astype(np.float32)
    eng = _eng(hp, syn.model._weights, 1, 2 * hop)
    out = eng.generate(cond, um, ul, 0, wav[None])
    eng.close()
    np.testing.assert_array_equal(got[0], out["y"][0])


def test_quantize_teacher_classes_validated():
    """a 'mulaw-quantize' teacher class outside [0, Q) (or not an integer) is refused on
    the host instead of indexing past the first conv's rows on the next sample."""
    from tt2._lib import TT2Error
    from tt2.weights import init_wavenet_weights
    hp = _quant_hp(6, 2)
    W = init_wavenet_weights(hp, seed=5339)
    B, T = 1, 275
    cond = WR.interp_condition(np.zeros((B, 1, 80), np.float32))
    _, ul = mol_uniforms(T, B, seed=4)
    eng = _eng(hp, W, B, T)
    try:
        for bad in (256.0, -1.0, 3.5):
            teacher = np.full((B, T), 7.0, np.float32)
            teacher[0, 100] = bad
            with pytest.raises(TT2Error, match="integer classes"):
                eng.generate(cond, None, ul, 0, teacher)
        out = eng.generate(cond, None, ul, 0, np.full((B, T), 255.0, np.float32))
        assert out["k"].shape == (B, T)
    finally:
        eng.close()
