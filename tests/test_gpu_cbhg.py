"""CBHG post-processing net + linear projection (modules.py:110-184; the reference's caller is
commented out at tacotron.py:466-481, VERDICT r01 missing item 7): libtt2 tt2_linear_outputs vs
oracle/tacotron_ref.py:linear_outputs within 1e-4, narrow and fork widths, and through
Tacotron.initialize with hp.predict_linear."""
import numpy as np
import pytest

from _common import full_hparams, oracle_hp, prenet_masks, small_hparams, tacotron_inputs
from oracle import tacotron_ref as TR

pytestmark = pytest.mark.gpu


def _hp(full):
    hp = full_hparams() if full else small_hparams()
    hp.predict_linear = True
    if not full:
        hp.override_from_dict(dict(cbhg_kernels=5, cbhg_conv_channels=32, cbhg_pool_size=3,
                                   cbhg_projection=48, cbhg_highwaynet_layers=2,
                                   cbhg_highway_units=32, cbhg_rnn_units=24, num_freq=97))
    return hp


def _ohp(hp):
    oh = oracle_hp(hp)
    oh.update({k: getattr(hp, k) for k in ("cbhg_kernels", "cbhg_pool_size", "cbhg_highway_units",
                                           "cbhg_highwaynet_layers")})
    return oh


@pytest.mark.parametrize("full", [False, True])
def test_linear_outputs(full):
    from tt2.engine import TacotronEngine
    from tt2.weights import init_tacotron_weights
    hp = _hp(full)
    W = init_tacotron_weights(hp, seed=5339)
    B, T = 2, 57
    mels = np.random.default_rng(8).uniform(-4, 4, (B, T, hp.num_mels)).astype(np.float32)
    eng = TacotronEngine(hp, W, B, 8, 64, 8)
    lin = eng.linear_outputs(mels)
    eng.close()
    ref = TR.linear_outputs(mels, W, _ohp(hp))
    assert lin.shape == (B, T, hp.num_freq)
    np.testing.assert_allclose(lin, ref, atol=1e-4)


def test_shim_predict_linear():
    from types import SimpleNamespace
    from tacotron.models import create_model
    hp = _hp(False)
    hp.override_from_dict(dict(max_iters=10))
    ids, lens, re, rs = tacotron_inputs(2, 9, 64, seed=15)
    masks = prenet_masks(10, 2, hp.prenet_layers[0], seed=15)
    m = create_model("Tacotron", hp)
    m.init_random_weights()
    m.initialize(SimpleNamespace(emt_only=False, synth_constraint=False), ids, lens, ref_mel_emt=re,
                 ref_mel_spk=rs, n_emt=4, n_spk=2, prenet_masks=masks)
    ref = TR.linear_outputs(m.tower_mel_outputs[0], m._weights, _ohp(hp))
    np.testing.assert_allclose(m.tower_linear_outputs[0], ref, atol=1e-4)
