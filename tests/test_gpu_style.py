"""Style paths of the Tacotron model besides GST (tacotron.py:236-308; VERDICT r01 missing item 6)
on the HIP library vs the oracle: 'embed' = args.pretrained_emb_disc_all (or hp.use_gst=False),
the reference embeddings concatenated into the memory (D_mem = 512 + 2x128), and 'adain' =
args.adain, ReferenceEncoderAdaIn over both references (modules.py:66-107, D_mem = 512 + 128).
Both widths: the narrow config decodes on the launch path, the fork widths on the persistent
decoder (the style only enters through the per-utterance GS / PS terms)."""
import numpy as np
import pytest

from _common import full_hparams, oracle_hp, prenet_masks, small_hparams, tacotron_inputs
from oracle import tacotron_ref as TR

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _run(hp, style, B=3, T=11, n=24, emt_only=False, seed=12):
    from tt2.engine import TacotronEngine
    from tt2.weights import init_tacotron_weights
    W = init_tacotron_weights(hp, seed=5339, emt_only=emt_only, style=style)
    ids, lens, re, rs = tacotron_inputs(B, T, 100, seed=seed)
    rs = None if emt_only else np.ascontiguousarray(rs[:, :72])
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=seed)
    eng = TacotronEngine(hp, W, B, T, 100, n, 0, emt_only, style=style)
    out = eng.synthesize(ids, lens, re, rs, n, masks)
    path, _ = eng.decoder_path()
    eng.close()
    oh = oracle_hp(hp, style=style)
    oh["emt_only"] = emt_only
    ref = TR.synthesize(ids, lens, re, rs, W, oh, masks, n)
    np.testing.assert_allclose(out["style"], ref["style"], atol=1e-5)
    np.testing.assert_allclose(out["encoder_outputs"], ref["encoder_outputs"], atol=1e-5)
    for k in ("stop_token_prediction", "alignments", "decoder_output", "mel_outputs"):
        np.testing.assert_allclose(out[k], ref[k], atol=TOL, err_msg=k)
    return path


@pytest.mark.parametrize("style", ["embed", "adain"])
def test_style_launch_path(style):
    assert _run(small_hparams(), style) == 0


@pytest.mark.parametrize("style", ["embed", "adain"])
def test_style_persistent_decoder(style):
    assert _run(full_hparams(), style, B=4, T=21, n=30) == 1


def test_embed_emt_only():
    _run(small_hparams(), "embed", emt_only=True)


def test_shim_adain_and_pretrained_emb_disc_all():
    from types import SimpleNamespace
    from tacotron.models import create_model
    hp = small_hparams()
    hp.override_from_dict(dict(max_iters=12))
    ids, lens, re, rs = tacotron_inputs(2, 9, 100, seed=14)
    masks = prenet_masks(12, 2, hp.prenet_layers[0], seed=14)
    for style, flags in (("adain", dict(adain=True)), ("embed", dict(pretrained_emb_disc_all=True))):
        args = SimpleNamespace(emt_only=False, synth_constraint=False, **flags)
        m = create_model("Tacotron", hp)
        m.init_random_weights(style=style)
        m.initialize(args, ids, lens, ref_mel_emt=re, ref_mel_spk=rs, n_emt=4, n_spk=2,
                     prenet_masks=masks)
        ref = TR.synthesize(ids, lens, re, rs, m._weights, oracle_hp(hp, style=style), masks, 12)
        np.testing.assert_allclose(m.tower_mel_outputs[0], ref["mel_outputs"], atol=TOL)
