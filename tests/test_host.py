"""CPU tests of the host side: hparams, weight key space, the C-ABI library (loads and exports
every symbol include/tt2.h declares — no compute calls without a GPU), shim validation that
mirrors the reference's argument checks, and the no-fallback rule."""
import argparse
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from _common import small_hparams
from tt2 import _lib
from tt2.hparams import HParams, bench_wavenet_hparams, get_hop_size, hparams, paper_hparams
from tt2.weights import (init_tacotron_weights, memory_width, tacotron_weight_specs,
                         wavenet_weight_specs)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tt2.h")


# ---------------------------------------------------------------- hparams
def test_hparams_parse_and_override():
    hp = hparams.copy()
    hp.parse("outputs_per_step=1,max_iters=123,prenet_layers=[128,128],stop_at_any=True")
    assert hp.max_iters == 123 and hp.prenet_layers == [128, 128] and hp.stop_at_any is True
    with pytest.raises(ValueError):
        hp.parse("no_such_param=3")
    assert hparams.max_iters == 1000      # copy() did not alias the defaults


def test_paper_hparams_backfill():
    # code/paper_hparams.py values for the WaveNet vocoder (24 layers / 4 stacks, MoL 10 mixtures)
    assert paper_hparams.layers == 24 and paper_hparams.stacks == 4
    assert paper_hparams.out_channels == 30 and paper_hparams.upsample_scales == [5, 5, 11]
    assert get_hop_size(paper_hparams) == 275
    # fork-only keys exist in the paper set (back-filled from code/hparams.py)
    assert paper_hparams.use_gst is True and paper_hparams.num_gst == 10
    b = bench_wavenet_hparams()
    assert (b.residual_channels, b.gate_channels, b.skip_out_channels) == (64, 128, 64)


def test_hparams_copy_independent():
    a = HParams(x=[1, 2])
    b = a.copy()
    b.x.append(3)
    assert a.x == [1, 2]


# ---------------------------------------------------------------- weights
def test_tacotron_weight_shapes_full():
    hp = hparams.copy()
    specs = {n: s for n, s, _ in tacotron_weight_specs(hp)}
    P = "Tacotron_model/inference/"
    D = memory_width(hp)
    # encoder outputs ⊕ emotion style ⊕ speaker style (tacotron.py:300-310); emt_only drops spk
    assert D == 2 * hp.encoder_lstm_units + 2 * hp.style_embed_depth
    assert memory_width(hp, emt_only=True) == 2 * hp.encoder_lstm_units + hp.style_embed_depth
    assert specs[P + "inputs_embedding"][1] == 512
    lstm0 = P + "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel"
    assert specs[lstm0] == (256 + D + 1024, 4096)     # [prenet ⊕ context ⊕ h, 4·units]
    lstm1 = P + "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/kernel"
    assert specs[lstm1] == (2048, 4096)
    proj = [n for n in specs if "linear_transform_projection" in n and n.endswith("kernel")]
    assert specs[proj[0]] == (1024 + D, 80)
    total = sum(int(np.prod(s)) for s in specs.values())
    assert 29e6 < total < 32e6


def test_wavenet_weight_specs_bench():
    hp = bench_wavenet_hparams()
    specs = {n: s for n, s, _ in wavenet_weight_specs(hp)}
    convs = [n for n in specs
             if re.search(r"ResidualConv1DGLU_\d+/residual_block_causal_conv_\w+/kernel$", n)]
    assert len(convs) == 24
    assert specs[convs[0]] == (3, 64, 128)
    total = sum(int(np.prod(s)) for s in specs.values())
    assert 0.9e6 < total < 1.2e6


def test_seeded_init_deterministic():
    hp = small_hparams()
    a = init_tacotron_weights(hp, seed=11)
    b = init_tacotron_weights(hp, seed=11)
    c = init_tacotron_weights(hp, seed=12)
    k = sorted(a)[3]
    np.testing.assert_array_equal(a[k], b[k])
    assert not np.array_equal(a[k], c[k])


# ---------------------------------------------------------------- the C ABI
def _header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(tt2_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert _header_symbols() == sorted(_lib.SIGNATURES)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "tacotron-2_amd"), "-j8"])
    return _lib.load_library()


def test_library_exports_every_header_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in _header_symbols() if s not in exported]
    assert not missing, missing
    assert lib.tt2_version().decode().startswith("libtt2")


def test_library_has_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob      # the offload bundle's target id


def test_config_struct_layout(lib):
    cfg = _lib.Config()
    lib.tt2_default_config(ctypes.byref(cfg), 4, 100, 200, 300)
    assert cfg.num_mels == 80 and cfg.decoder_lstm_units == 1024 and cfg.prenet_units == 256
    assert (cfg.max_batch, cfg.max_T_in, cfg.max_T_ref, cfg.max_iters) == (4, 100, 200, 300)
    assert list(cfg.reference_filters) == [32, 32, 64, 64, 128, 128]
    w = _lib.WnConfig()
    lib.tt2_wn_default_config(ctypes.byref(w), 2, 22050)
    assert w.max_batch == 2 and w.max_samples == 22050 and w.out_channels == 30


def test_create_without_gpu_fails_loudly(lib):
    """No CPU fallback: on a GPU-less host tt2_create returns HIP_ERROR with a message."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    cfg = _lib.Config()
    lib.tt2_default_config(ctypes.byref(cfg), 1, 8, 8, 8)
    h = ctypes.c_void_p()
    st = lib.tt2_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert st == -4 and not h.value
    assert b"hip" in lib.tt2_last_error().lower()
    with pytest.raises(_lib.TT2Error):
        _lib.check(st)


def test_create_rejects_bad_config(lib):
    cfg = _lib.Config()
    lib.tt2_default_config(ctypes.byref(cfg), 0, 8, 8, 8)   # max_batch 0
    h = ctypes.c_void_p()
    assert lib.tt2_create(ctypes.byref(cfg), 0, ctypes.byref(h)) != 0
    assert not h.value


def test_missing_library_raises(tmp_path):
    saved = _lib._lib
    _lib._lib = None
    try:
        with pytest.raises(_lib.TT2NotBuilt):
            _lib.load_library(str(tmp_path / "libtt2.so"))
    finally:
        _lib._lib = saved


# ---------------------------------------------------------------- reference-API shims
def _args(**kw):
    d = dict(emt_only=False, adain=False, unpaired=False, pretrained_emb_disc_all=False,
             synth_constraint=False, nat_gan=False)
    d.update(kw)
    return argparse.Namespace(**d)


def _taco():
    from tacotron.models import create_model
    hp = small_hparams()
    return create_model("Tacotron", hp), hp


def test_create_model_names():
    from tacotron.models import create_model
    with pytest.raises(Exception, match="Unknown model"):
        create_model("Nope", small_hparams())
    from tacotron.models import Tacotron_emt_attn
    assert isinstance(create_model("Tacotron_emt_attn", small_hparams()), Tacotron_emt_attn)


@pytest.mark.parametrize("kw,exc", [
    (dict(stop_token_targets=np.zeros((1, 3))), ValueError),                   # tacotron.py:48
    (dict(mel_targets=np.zeros((1, 3, 80))), ValueError),                      # tacotron.py:50
    (dict(gta=True, mel_targets=np.zeros((1, 3, 80)), linear_targets=np.zeros(1)), ValueError),
    (dict(is_training=True, is_evaluating=True, targets_lengths=[3]), RuntimeError),
    (dict(ref_mel_emt=None), ValueError),                                      # references
])
def test_tacotron_initialize_validation(kw, exc):
    m, hp = _taco()
    base = dict(inputs=np.ones((1, 5), np.int32), input_lengths=[5],
                ref_mel_emt=np.zeros((1, 20, 80), np.float32),
                ref_mel_spk=np.zeros((1, 20, 80), np.float32), n_emt=4, n_spk=4)
    base.update(kw)
    with pytest.raises(exc):
        m.initialize(_args(), **base)


def test_tacotron_needs_weights_before_engine():
    m, hp = _taco()
    with pytest.raises(RuntimeError, match="weights not loaded"):
        m.initialize(_args(), np.ones((1, 5), np.int32), [5], ref_mel_emt=np.zeros((1, 20, 80)),
                     ref_mel_spk=np.zeros((1, 20, 80)), n_emt=4, n_spk=4)


def test_tacotron_training_needs_style_labels():
    """is_training=True is built (tests/test_gpu_train_api.py); the default graph's style-embedding
    classifiers need the labels, refused before any device work."""
    m, hp = _taco()
    with pytest.raises(ValueError, match="emt_labels"):
        m.initialize(_args(), np.ones((1, 5), np.int32), [5], mel_targets=np.zeros((1, 3, 80)),
                     stop_token_targets=np.zeros((1, 3)), targets_lengths=[3], is_training=True,
                     ref_mel_emt=np.zeros((1, 20, 80)), ref_mel_spk=np.zeros((1, 20, 80)),
                     n_emt=4, n_spk=4)


def test_split_func_matches_reference_packing():
    from tacotron.models.tacotron import split_func
    x = np.arange(2 * 7).reshape(2, 7)
    a, b = split_func(x, np.array([3, 4]))
    np.testing.assert_array_equal(a, x[:, :3])
    np.testing.assert_array_equal(b, x[:, 3:])


def test_wavenet_shim_scope_checks():
    from wavenet_vocoder.models import create_model
    hp = bench_wavenet_hparams()
    m = create_model("WaveNet", hp)
    assert m.receptive_field == 505
    assert m.local_conditioning_enabled()
    with pytest.raises(RuntimeError, match="weights not loaded"):
        m.initialize(None, np.zeros((1, 2, 80), np.float32), None, None, synthesis_length=None)
    hp2 = bench_wavenet_hparams().override_from_dict(dict(gin_channels=16))  # global conditioning
    with pytest.raises(ValueError, match="global condition"):                 # ... needs g
        create_model("WaveNet", hp2).initialize(None, np.zeros((1, 2, 80), np.float32), None, None)


def test_mixture_shim_validates_channels():
    from wavenet_vocoder.models.mixture import sample_with_index
    with pytest.raises(ValueError):
        sample_with_index(np.zeros((1, 31, 4), np.float32))


def test_product_does_not_import_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline may touch oracle/."""
    pkg = os.path.join(ROOT, "tacotron-2_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f


def test_oracle_output_lengths_and_condition_batch():
    from oracle import tacotron_ref as TR
    from oracle import wavenet_ref as WR
    stop = np.array([[0.1, 0.5, 0.51, 0.9], [0.2, 0.2, 0.3, 0.4], [0.7, 0.1, 0.1, 0.1]], np.float32)
    assert TR.get_output_lengths(stop) == [2, 4, 0]
    m = [np.full((3, 80), 5.0, np.float32), np.full((1, 80), -1.0, np.float32)]
    c = WR.condition_batch(m)
    assert c.shape == (2, 3, 80)
    np.testing.assert_array_equal(c[0], 1.0)                 # clipped to 4 -> 1
    np.testing.assert_array_equal(c[1, 0], 3.0 / 8.0)        # (-1 + 4) / 8
    np.testing.assert_array_equal(c[1, 1:], 0.0)             # padded with -4 -> 0


def test_synthesizer_filenames_to_inputs_pads_per_tower(tmp_path):
    """tacotron/synthesizer.py:296-371: ids padded with 0 per tower and concatenated on the time
    axis, reference mels padded with -max_abs_value, split_infos [max_seq_len,0,0,0,0,T_e,T_s]."""
    from tacotron.synthesizer import filenames_to_inputs, get_output_lengths
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=2, tacotron_synthesis_batch_size=2))
    refs = [np.ones((5 + i, 80), np.float32) for i in range(4)]
    out = filenames_to_inputs(hp, ["ab", "abcd", "a", "abc"], ["b0", "b1", "b2", "b3"], None,
                              ["r"] * 4, refs, refs[::-1])
    _, _, seqs, lens, split, re, rs, _, _ = out
    np.testing.assert_array_equal(lens, [3, 5, 2, 4])
    assert seqs.shape == (2, 5 + 4)
    np.testing.assert_array_equal(split[:, 0], [5, 4])
    np.testing.assert_array_equal(split[:, 5], [6, 8])
    assert re.shape == (2, 6 + 8, 80) and rs.shape == (2, 8 + 6, 80)
    assert re[0, 5, 0] == -4.0 and re[1, 6 + 7, 0] == 1.0
    assert get_output_lengths(np.array([[0.2, 0.7], [0.1, 0.1]])) == [1, 2]


def test_wavenet_synthesizer_host_prep_and_conditions():
    """The Synthesizer's host prep (_interp) and its condition switches: cin_channels <= 0 builds the
    unconditional synthesis_length path (synthesizer.py:51-53,75-78), wavenet_synth_debug needs the
    debug mels and wavs to pair up (synthesizer.py:56-58)."""
    from wavenet_vocoder.synthesizer import SYNTHESIS_LENGTH, Synthesizer, _interp
    np.testing.assert_allclose(_interp(np.array([-4.0, 0.0, 4.0]), (-4, 4)), [0, 0.5, 1])
    hp = bench_wavenet_hparams()
    hp.cin_channels = -1
    syn = Synthesizer()
    syn.load(None, hp)
    assert syn._check_conditions() == (False, False) and SYNTHESIS_LENGTH == 100
    hp = bench_wavenet_hparams()
    hp.override_from_dict(dict(wavenet_synth_debug=True, wavenet_debug_mels=["a.npy", "b.npy"],
                               wavenet_debug_wavs=["a.npy"]))
    syn = Synthesizer()
    syn.load(None, hp)
    with pytest.raises(ValueError, match="pair up"):
        syn.synthesize([np.zeros((2, 80), np.float32)], None, ["x"], None, None)


def test_wavenet_gc_weight_specs():
    """gin_channels > 0 adds conv1x1g to every layer (modules.py:427-433) and, with
    use_speaker_embedding, the gc_embedding table (wavenet.py:152-156); off by default."""
    from tt2.weights import wavenet_weight_specs
    hp = bench_wavenet_hparams()
    names = [n for n, _, _ in wavenet_weight_specs(hp)]
    assert not any("gin_conv" in n or "gc_embedding" in n for n in names)
    hp.gin_channels, hp.use_speaker_embedding, hp.n_speakers = 16, True, 7
    specs = {n: s for n, s, _ in wavenet_weight_specs(hp)}
    k = "WaveNet_model/inference/ResidualConv1DGLU_3/residual_block_gin_conv_ResidualConv1DGLU_3/kernel"
    assert specs[k] == (1, 16, hp.gate_channels)
    assert specs["WaveNet_model/gc_embedding"] == (7, 16)


@pytest.mark.parametrize("src,kernel,max_spill", [("wavenet.hip", "k_generate_pipe", 0),
                                                  ("decode_persist.hip", "k_decode_persistILb0", 32),
                                                  ("decode_persist.hip", "k_decode_persistILb1", 96)])
def test_register_resident_kernels_do_not_spill(src, kernel, max_spill):
    """The WaveNet generator keeps its weights in registers: a VGPR spill on its per-sample chain
    cost 19 % (23 spills from a runtime head flag, fixed by a template parameter) — guard it at
    build time with the compiler's resource-usage remarks (no GPU needed).  The persistent decoder
    spills 21 VGPRs by measurement-driven choice: its spill-free variants (constants moved to
    LDS) were 1.5-2.5 % slower (28.9 / 29.2 vs 28.5 us/step) because the reloads sit off the
    critical path; the bound keeps it from growing.  The Tacotron_emt_attn instantiation
    (k_decode_persist<true>, round 3) carries the emotion stages on top and has its own bound."""
    import shutil
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    pkg = os.path.join(ROOT, "tacotron-2_amd")
    r = subprocess.run([hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c",
                        os.path.join(pkg, "csrc", src), "-o", os.devnull,
                        "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    blocks = r.stderr.split("Function Name: ")[1:]
    mine = [b for b in blocks if kernel in b.splitlines()[0]]
    assert mine, "no resource-usage remarks for " + kernel
    for b in mine:
        spill = re.search(r"VGPRs Spill: (\d+)", b)
        assert spill and int(spill.group(1)) <= max_spill, b.splitlines()[0] + " spills VGPRs"


def test_mulaw_companding_matches_reference_formulas():
    """wavenet_vocoder/util.py:29-127 (mu fixed at 255 whatever the argument): known values and
    round trips of mulaw / inv_mulaw / mulaw_quantize / inv_mulaw_quantize."""
    import numpy as np
    from wavenet_vocoder.util import inv_mulaw, inv_mulaw_quantize, mulaw, mulaw_quantize
    assert mulaw(0.0) == 0.0 and abs(mulaw(1.0) - 1.0) < 1e-12 and abs(mulaw(-1.0) + 1.0) < 1e-12
    assert mulaw_quantize(0.0) == 127 and mulaw_quantize(1.0) == 255 and mulaw_quantize(-1.0) == 0
    x = np.linspace(-1, 1, 1001)
    np.testing.assert_allclose(inv_mulaw(mulaw(x)), x, atol=1e-12)
    np.testing.assert_allclose(mulaw(0.5), np.log1p(127.5) / np.log1p(255.0), rtol=1e-12)
    np.testing.assert_allclose(mulaw(0.5, mu=65536), mulaw(0.5))
    q = mulaw_quantize(x)
    assert q.min() == 0 and q.max() == 255
    assert np.abs(inv_mulaw_quantize(q) - x).max() < 0.05
