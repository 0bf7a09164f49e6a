"""GPU parity of the end-to-end text -> mel -> wav path (BASELINE.json configs[3]).

Pieces: ``tt2_output_lengths_dev`` (get_output_lengths, tacotron/synthesizer.py:384-387),
``tt2_wn_cond_from_mels_dev`` (wavenet_vocoder/synthesizer.py:52-70), ``tt2.e2e.TextToSpeech``
(both models with the mel hand-off in HBM) and the reference-named ``Synthesizer`` shims with their
``mel-*.npy`` / ``.wav`` file contract.  Oracle: oracle/tacotron_ref.py + oracle/wavenet_ref.py.
Tolerances as in test_gpu_parity.py: mels 1e-4; stop lengths exact; conditioning 1e-6 (one fp32
rounding of the rescale); MoL indices exact on a free-running prefix of >= 200 samples.
"""
import ctypes

import numpy as np
import pytest

from _common import mol_uniforms, oracle_hp, prenet_masks, wavenet_oracle_hp
from oracle import tacotron_ref as TR
from oracle import wavenet_ref as WR

pytestmark = pytest.mark.gpu

SMALL_TACO = dict(embedding_dim=64, enc_conv_channels=64, encoder_lstm_units=32, attention_dim=32,
                  attention_filters=8, prenet_layers=[32, 32], decoder_lstm_units=64,
                  postnet_channels=64, style_embed_depth=64, style_att_dim=32,
                  reference_filters=[8, 8, 16, 16, 32, 32], reference_depth=32)


def _lib():
    from tt2 import _lib as L
    return L, L.load_library()


def test_output_lengths_kernel():
    import torch
    L, lib = _lib()
    n, ld = 150, 160
    rng = np.random.default_rng(3)
    stop = rng.uniform(0, 0.49, (7, ld)).astype(np.float32)
    stop[1, 0] = 0.9            # stops at step 0
    stop[2, 64] = 0.5           # exactly one half rounds to 0 (half to even) ...
    stop[2, 65] = 0.50000006    # ... the next float up rounds to 1
    stop[3, 149] = 1.0          # last decoded step
    stop[4, 150] = 1.0          # past n_steps: ignored
    stop[5, 10] = stop[5, 90] = 0.7  # first occurrence wins
    stop[6, 63] = 0.8           # wave-chunk boundary
    d = torch.from_numpy(stop).cuda()
    out = torch.empty(7, dtype=torch.int32, device="cuda")
    L.check(lib.tt2_output_lengths_dev(d.data_ptr(), 7, n, ld, out.data_ptr(),
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    got = out.cpu().numpy().tolist()
    assert got == TR.get_output_lengths(stop[:, :n])
    assert got == [150, 0, 65, 149, 150, 10, 63]


@pytest.mark.parametrize("T_f,lens", [(37, [37, 5, 0, 33]), (1, [1, 1]), (100, [64, 100, 99])])
def test_cond_from_mels_kernel(T_f, lens):
    import torch
    L, lib = _lib()
    B, n, F = len(lens), 110, 80
    rng = np.random.default_rng(T_f)
    mels = rng.uniform(-5, 5, (B, n, F)).astype(np.float32)  # beyond [-4, 4]: exercises the clip
    lens_a = np.asarray(lens, np.int32)
    md = torch.from_numpy(mels).cuda()
    ld = torch.from_numpy(lens_a).cuda()
    cond = torch.full((B, F, T_f), np.nan, dtype=torch.float32, device="cuda")
    L.check(lib.tt2_wn_cond_from_mels_dev(md.data_ptr(), n, ld.data_ptr(), B, T_f, F, -4.0, 4.0, 1,
                                          1, cond.data_ptr(),
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    got = cond.cpu().numpy()
    # condition_batch pads to the longest mel; pad the reference list to T_f with one dummy row
    ref = WR.condition_batch([mels[b, :lens[b]] for b in range(B)] + [np.zeros((T_f, F), np.float32)])
    np.testing.assert_allclose(got, ref[:B].transpose(0, 2, 1), rtol=0, atol=1e-6)


def _e2e_hp(n):
    from tt2.e2e import e2e_hparams
    hp = e2e_hparams(n)
    hp.override_from_dict(dict(SMALL_TACO))
    return hp


def test_e2e_text_to_wav_matches_oracle():
    """texts -> ids (text frontend) -> Tacotron (mels, stop) -> lengths -> WaveNet conditioning ->
    24-layer MoL WaveNet, all on the device; every stage against the oracle."""
    from tacotron.utils.text import text_to_sequence
    from tt2.e2e import TextToSpeech
    from tt2.weights import init_tacotron_weights, init_wavenet_weights
    n = 5
    hp = _e2e_hp(n)
    W = init_tacotron_weights(hp, seed=5339)
    # stop bias low enough that no row stops within n steps: every row keeps n frames, so the
    # WaveNet leg runs over a known length (ragged lengths are covered by the kernel tests)
    W["Tacotron_model/inference/decoder/stop_token_projection/projection_stop_token_projection/"
      "bias"] = np.full((1,), -6.0, np.float32)
    WW = init_wavenet_weights(hp, seed=5339)
    texts = ["Turn left at 21 Baker St.", "It costs $3.50, Dr. Who said."]
    seqs = [text_to_sequence(t, ["english_cleaners"]) for t in texts]
    B, T_in = len(seqs), max(len(s) for s in seqs)
    ids = np.zeros((B, T_in), np.int32)
    for b, s in enumerate(seqs):
        ids[b, :len(s)] = s
    lens = np.asarray([len(s) for s in seqs], np.int32)
    rng = np.random.default_rng(11)
    re = rng.uniform(-4, 4, (B, 48, 80)).astype(np.float32)
    rs = rng.uniform(-4, 4, (B, 48, 80)).astype(np.float32)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=4)
    T = n * hp.hop_size
    um, ul = mol_uniforms(T, B, seed=9)
    tts = TextToSpeech(hp, W, WW, B, T_in, 48, n, 0)
    out = tts.synthesize(ids, lens, re, rs, 0, um, ul, masks)
    tts.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    np.testing.assert_allclose(out["mel"], ref["mel_outputs"], atol=1e-4)
    assert list(out["lengths"]) == TR.get_output_lengths(ref["stop_token_prediction"])
    assert out["n_steps"] == n
    # WaveNet leg from the device mels (isolates the hand-off + vocoder from 1e-5 mel noise)
    mels = [out["mel"][b, :out["lengths"][b]] for b in range(B)]
    cond = WR.condition_batch(mels)
    c_up = WR.upsample_2d(cond.transpose(0, 2, 1), WW, hp.upsample_scales)
    y, k = WR.incremental(c_up.transpose(0, 2, 1), WW, wavenet_oracle_hp(hp), um, ul)
    for b in range(B):
        assert out["wavs"][b].shape == (out["lengths"][b] * hp.hop_size,)
        # free running: identical until a (rare) near-tie diverges
        kk = np.asarray(out["wavs"][b])
        same = np.abs(kk - y[b, :kk.shape[0]]) < 1e-4
        first = int(np.argmin(same)) if not same.all() else kk.shape[0]
        assert first >= 200, (b, first)


def test_synthesizer_file_contract(tmp_path):
    """tacotron.synthesizer.Synthesizer writes mel-<base>_<ref>.npy files trimmed by the stop
    tokens and clipped to [-4, 4]; wavenet_vocoder.synthesizer.Synthesizer turns them into
    wavenet-audio-<base>.wav of T_i * hop samples (the two halves of code/synthesize.py:33-43)."""
    from types import SimpleNamespace

    from scipy.io import wavfile

    from tacotron.synthesizer import Synthesizer as TacoSynth
    from wavenet_vocoder.synthesizer import Synthesizer as WnSynth
    n = 6
    hp = _e2e_hp(n)
    hp.override_from_dict(dict(layers=6, stacks=2))
    rng = np.random.default_rng(2)
    refs = []
    for i in range(2):
        p = str(tmp_path / "ref{}.npy".format(i))
        np.save(p, rng.uniform(-4, 4, (40 + 7 * i, 80)).astype(np.float32))
        refs.append(p)
    args = SimpleNamespace(emt_attn=False, attn="style_tokens", emt_only=False)
    ts = TacoSynth()
    ts.load(args, None, hp)
    texts = ["Hello world.", "A second, longer sentence with 42 words?"]
    paths, spk = ts.synthesize(texts, ["a", "b"], str(tmp_path), str(tmp_path), None,
                               basenames_refs=["r0", "r1"], mel_ref_filenames_emt=refs,
                               mel_ref_filenames_spk=refs[::-1],
                               prenet_masks=prenet_masks(n, 2, hp.prenet_layers[0], seed=1))
    assert [p.split("/")[-1] for p in paths] == ["mel-a_r0.npy", "mel-b_r1.npy"]
    for b, r in (("a", "r0"), ("b", "r1")):   # Griffin-Lim wavs of the eval log dir
        sr, gl = wavfile.read(str(tmp_path / "wavs" / "wav-{}_{}.wav".format(b, r)))
        assert sr == hp.sample_rate and gl.dtype == np.int16
    assert spk == ["<no_g>", "<no_g>"]
    mels = [np.load(p, allow_pickle=False) for p in paths]
    for m, tl in zip(mels, ts.target_lengths):
        assert m.shape == (tl, 80) and m.dtype == np.float32
        assert np.all(np.abs(m) <= 4.0)
    ws = WnSynth()
    ws.load(None, hp)
    keep = [m for m in mels if len(m)]
    if not keep:
        pytest.skip("random-weight Tacotron stopped at step 0 on every row")
    wavs = ws.synthesize(keep, None, ["a", "b"][:len(keep)], str(tmp_path / "wavs"), None)
    for w, m in zip(wavs, keep):
        sr, data = wavfile.read(w)
        assert sr == hp.sample_rate and data.dtype == np.int16
        assert data.shape == (len(m) * hp.hop_size,)


def test_configs3_fork_widths_product_chain_matches_oracle():
    """configs[3]'s product chain at the fork-default widths: text frontend ->
    encoder -> the PERSISTENT decoder (k_decode_persist; D_mem 1024, 2 x 1024 LSTM) -> Postnet ->
    tt2_output_lengths_dev -> tt2_wn_cond_from_mels_dev -> 24-layer R=64 MoL WaveNet
    (k_generate_pipe), all on one stream through TextToSpeech.synthesize, B=3 utterances of 136-201
    characters, 60 decoder steps, 16,500 samples per row.  Checks: mels within 1e-4 of the oracle,
    lengths exact, conditioning within 1e-6 of condition_batch on the device mels, the free-running
    waveform identical to the oracle's on a >= 200-sample prefix, and along the device's own
    trajectory (its waveform fed back as the teacher) logits within 1e-4 and mixture indices exact
    wherever the oracle's top-2 Gumbel margin exceeds 1e-4.
    Reference chain: synthesize.py:33-43, tacotron/synthesizer.py:186-189,384-387,
    wavenet_vocoder/synthesizer.py:56-70."""
    from _common import fork_e2e_case
    from tt2.e2e import TextToSpeech
    from tt2.engine import WaveNetEngine
    n = 60
    hp, W, WW, ids, lens, re, rs, masks, um, ul = fork_e2e_case(n)
    B, T_in = ids.shape
    assert T_in == 201 and hp.decoder_lstm_units == 1024
    tts = TextToSpeech(hp, W, WW, B, T_in, re.shape[1], n, 0)
    out = tts.synthesize(ids, lens, re, rs, 0, um, ul, masks)
    assert tts.taco.decoder_path()[0] == 1          # the persistent decoder served it
    tts.close()
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)
    assert out["n_steps"] == n
    np.testing.assert_allclose(out["mel"], ref["mel_outputs"], atol=1e-4)
    assert list(out["lengths"]) == TR.get_output_lengths(ref["stop_token_prediction"]) == [n] * B
    mels = [out["mel"][b, :out["lengths"][b]] for b in range(B)]
    cond = WR.condition_batch(mels)                 # [B, T_f, 80]
    np.testing.assert_allclose(out["cond"], cond.transpose(0, 2, 1), rtol=0, atol=1e-6)
    c_up = WR.upsample_2d(cond.transpose(0, 2, 1), WW, hp.upsample_scales).transpose(0, 2, 1)
    whp = wavenet_oracle_hp(hp)
    y, k = WR.incremental(c_up, WW, whp, um, ul)
    T = n * hp.hop_size
    dev_y = np.stack(out["wavs"])
    assert dev_y.shape == (B, T)
    for b in range(B):
        same = np.abs(dev_y[b] - y[b]) < 1e-4
        first = int(np.argmin(same)) if not same.all() else T
        assert first >= 200, (b, first)
    # the whole length along the device's trajectory: teacher = the device's free-run waveform
    eng = WaveNetEngine(hp, WW, B, T, 0)
    tf = eng.generate(cond, um, ul, 0, dev_y, want_logits=True)
    eng.close()
    yo, ko, lo = WR.incremental(c_up, WW, whp, um, ul, dev_y, return_logits=True)
    np.testing.assert_allclose(tf["logits"], lo, atol=1e-4, rtol=1e-4)
    gl = np.log(-np.log(um.astype(np.float64))).astype(np.float32)
    temp = lo[..., :10] - gl.transpose(1, 0, 2)
    srt = np.sort(temp, -1)
    safe = (srt[..., -1] - srt[..., -2]) > 1e-4
    assert safe.mean() > 0.99
    np.testing.assert_array_equal(tf["k"][safe], ko[safe])
    np.testing.assert_allclose(tf["y"][safe], yo[safe], atol=1e-4)
