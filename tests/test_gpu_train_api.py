"""The training step behind the reference's own training API (tacotron/train.py:104-139,
411-416): ``Tacotron.initialize(..., is_training=True)`` -> ``add_loss()`` ->
``add_optimizer(global_step)`` drives tt2.train.TacotronTrainer, and the teacher-forcing ratio
schedule is applied by the trainer itself (TacoTrainingHelper, helpers.py:99-131)."""
import types

import numpy as np
import pytest

from _common import small_hparams
from tt2.synthetic import (enc_conv_masks, enc_zoneout_masks, postnet_masks, prenet_masks, tacotron_inputs,
                           train_batch, zoneout_masks)
from tt2.weights import init_tacotron_weights, memory_width

ARGS = types.SimpleNamespace(adain=False, emt_only=False, unpaired=False, pretrained_emb_disc_all=False,
                             synth_constraint=False, nat_gan=False)


def _batch(hp, B=3, T_in=9, T_out=6, T_ref=70, seed=32):
    ids, lens, re, rs = tacotron_inputs(B, T_in, T_ref, seed=seed)
    _, _, tg, st = train_batch(B, T_in, T_out, memory_width(hp), seed=seed)
    m = dict(prenet=prenet_masks(T_out, B, hp.prenet_layers[0], seed=seed),
             zoneout=zoneout_masks(T_out, B, hp.decoder_lstm_units, seed=seed),
             postnet=postnet_masks(hp.postnet_num_layers, B, T_out, hp.postnet_channels, seed=seed),
             enc_conv=enc_conv_masks(hp.enc_conv_num_layers, B, T_in, hp.enc_conv_channels, seed=seed),
             enc_zoneout=enc_zoneout_masks(T_in, B, hp.encoder_lstm_units, seed=seed))
    return ids, lens, re, rs, tg, st, m


def _hp():
    hp = small_hparams()
    hp.override_from_dict(dict(tacotron_use_style_emb_disc=False, tacotron_use_orthog_loss=False))
    return hp


def _model(hp, W):
    from tacotron.models import create_model
    model = create_model("Tacotron", hp)
    model.load_weights(W)
    return model


def test_training_api_validation():
    """Refusals that need no GPU: eval graphs, unbuilt style paths, towers in one process,
    missing targets (tacotron.py:48-71 and the build's scope)."""
    hp = _hp()
    W = init_tacotron_weights(hp, seed=5339)
    ids, lens, re, rs, tg, st, _ = _batch(hp)
    model = _model(hp, W)
    with pytest.raises(NotImplementedError, match="eval"):
        model.initialize(ARGS, ids, lens, tg, st, is_evaluating=True, ref_mel_emt=re, ref_mel_spk=rs)
    with pytest.raises(ValueError, match="without corresponding token_targets"):
        model.initialize(ARGS, ids, lens, tg, None, is_training=True, ref_mel_emt=re, ref_mel_spk=rs)
    with pytest.raises(ValueError, match="AdaIn"):  # tacotron.py:68-69
        model.initialize(types.SimpleNamespace(**dict(vars(ARGS), adain=True, emt_only=True)), ids, lens, tg, st,
                         is_training=True, ref_mel_emt=re, ref_mel_spk=rs)
    hp3 = small_hparams()   # the default graph's style classifiers need the classes and labels
    with pytest.raises(ValueError, match="number of emotions"):
        _model(hp3, W).initialize(ARGS, ids, lens, tg, st, is_training=True, ref_mel_emt=re, ref_mel_spk=rs)
    with pytest.raises(ValueError, match="emt_labels"):
        _model(hp3, W).initialize(ARGS, ids, lens, tg, st, is_training=True, ref_mel_emt=re, ref_mel_spk=rs,
                                  n_emt=4, n_spk=3)
    hp2 = hp.copy()
    hp2.override_from_dict(dict(tacotron_num_gpus=3))
    with pytest.raises(NotImplementedError, match="one process per GPU"):
        _model(hp2, W).initialize(ARGS, ids, lens, tg, st, is_training=True, ref_mel_emt=re, ref_mel_spk=rs)
    with pytest.raises(RuntimeError, match="initialize"):
        _model(hp, W).add_loss()


@pytest.mark.gpu
@pytest.mark.parametrize("style", [False, True])
def test_reference_named_calls_match_trainer_step(style):
    """Two steps through initialize(is_training=True) / add_loss() / add_optimizer(global_step)
    equal TacotronTrainer.step_text on the same inputs and keep bits bit for bit: losses, the
    updated parameters of every training variable, decoder outputs; mel_outputs =
    clip(decoder_output + Postnet projection)."""
    from oracle import train_ref as TRN
    from tt2.train import TacotronTrainer, init_style_disc_weights
    hp = small_hparams() if style else _hp()   # style: the default graph's classifier + orthogonality losses
    W = init_tacotron_weights(hp, seed=5339)
    ne, ns = (4, 3) if style else (0, 0)
    W.update(init_style_disc_weights(hp, ne, ns, seed=3))
    el, sl = np.array([1, 3, 0], np.int32), np.array([2, 0, 1], np.int32)
    ids, lens, re, rs, tg, st, m = _batch(hp)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    model = _model(hp, W)
    got = []
    for step in range(2):
        model.initialize(ARGS, ids, lens, tg, st, is_training=True, ref_mel_emt=re, ref_mel_spk=rs, train_masks=m,
                         n_emt=ne or None, n_spk=ns or None, emt_labels=el, spk_labels=sl)
        loss = model.add_loss()
        gs = model.add_optimizer(step)
        assert gs == step + 1 and model.optimize == step + 1
        if style:
            assert model.style_emb_loss_emt > 0 and model.style_emb_loss_spk > 0 and model.style_emb_orthog_loss > 0
        got.append(dict(loss=loss, before=model.before_loss, after=model.after_loss, stop=model.stop_token_loss,
                        reg=model.regularization_loss, dec=model.tower_decoder_output[0].copy(),
                        mel=model.tower_mel_outputs[0].copy(), stop_logits=model.tower_stop_token_prediction[0].copy()))
    names = (TRN.frontend_var_names() + TRN.style_disc_var_names(False, ne, ns) + TRN.train_var_names()
             + TRN.postnet_var_names())
    params = {n: model._trainer.get(n, 0, np.asarray(W[n]).shape) for n in names}
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1], n_emt=ne, n_spk=ns)
    try:
        if style:
            tr.set_style_labels(el, sl)
        for step in range(2):
            L = tr.step_text(ids, lens, re, rs, tg, st, m["prenet"], m["zoneout"], m["postnet"], m["enc_conv"],
                             m["enc_zoneout"])
            fr, sl, _ = tr.outputs(T_in, T_out)
            g = got[step]
            assert g["loss"] == L["loss"] and g["before"] == L["before"] and g["after"] == L["after"]
            assert g["stop"] == L["stop_token"] and g["reg"] == L["regularization"]
            assert np.array_equal(g["dec"], fr) and np.array_equal(g["stop_logits"], sl)
            proj = tr.get("postnet:projection", 0, fr.shape)
            lo, hi = tr.cfg.clip_lo, tr.cfg.clip_hi
            np.testing.assert_array_equal(g["mel"], np.clip(fr + proj, lo, hi))
        for n in names:
            assert np.array_equal(params[n], tr.get(n, 0, params[n].shape)), n
        assert any(not np.array_equal(params[n], np.asarray(W[n], np.float32)) for n in names)
    finally:
        tr.close()
    tw = model.trained_weights()
    assert np.array_equal(tw[names[0]], params[names[0]])
    model._trainer.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["constant", "scheduled"])
def test_trainer_applies_teacher_forcing_schedule(mode):
    """a ratio below 1 ('constant') or the 'scheduled' decay is applied by the trainer
    itself -- the ratio at the global step before the update and one draw per decoder step from
    the trainer's seeded generator -- and equals injecting the same draw explicitly."""
    from tt2.train import TacotronTrainer, draw_teacher_forcing, teacher_forcing_ratio
    hp = _hp()
    if mode == "constant":
        hp.override_from_dict(dict(tacotron_teacher_forcing_ratio=0.5))
    else:
        hp.override_from_dict(dict(tacotron_teacher_forcing_mode="scheduled", tacotron_teacher_forcing_init_ratio=1.0,
                                   tacotron_teacher_forcing_start_decay=1, tacotron_teacher_forcing_decay_steps=1,
                                   tacotron_teacher_forcing_decay_exp_rate=0.5))
    W = init_tacotron_weights(hp, seed=5339)
    ids, lens, re, rs, tg, st, m = _batch(hp, T_out=8)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    args = (ids, lens, re, rs, tg, st, m["prenet"], m["zoneout"], m["postnet"], m["enc_conv"], m["enc_zoneout"])
    auto = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1], tf_seed=7)
    inj = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1])
    rng = np.random.default_rng(7)
    try:
        fed_own = 0
        for step in range(3):
            La = auto.step_text(*args)
            ratio = teacher_forcing_ratio(step, hp)
            assert auto.ratio == ratio
            feed = None if ratio >= 1.0 else draw_teacher_forcing(T_out, ratio, rng)
            fed_own += 0 if feed is None else int((feed == 0).sum())
            inj.set_step_inputs(feed_target=feed)
            Li = inj.step_text(*args)
            assert La["loss"] == Li["loss"] and La["grad_norm"] == Li["grad_norm"], step
        assert fed_own > 0   # the draw did feed predicted frames somewhere
    finally:
        auto.close()
        inj.close()


@pytest.mark.gpu
def test_style_classifier_variables_saved_and_restored():
    """the Style_Emb_Disc variables the trainer draws fresh (the loaded weights lack
    them) are part of the saved weights after training, and a model resumed from those weights
    trains from the saved values, not a re-drawn initialisation (tf.train.Saver round trip)."""
    from oracle import train_ref as TRN
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    ne, ns = 4, 3
    names = TRN.style_disc_var_names(False, ne, ns)
    assert names and not any(n in W for n in names)
    el, sl = np.array([1, 3, 0], np.int32), np.array([2, 0, 1], np.int32)
    ids, lens, re, rs, tg, st, m = _batch(hp)
    kw = dict(is_training=True, ref_mel_emt=re, ref_mel_spk=rs, train_masks=m, n_emt=ne, n_spk=ns,
              emt_labels=el, spk_labels=sl)
    model = _model(hp, W)
    model.initialize(ARGS, ids, lens, tg, st, **kw)
    model.add_loss()
    model.add_optimizer(0)
    assert all(n in model.all_vars for n in names)
    saved = model.trained_weights()
    trained = {n: model._trainer.get(n, 0, saved[n].shape) for n in names}
    model._trainer.close()
    for n in names:
        np.testing.assert_array_equal(saved[n], trained[n])
    resumed = _model(hp, saved)
    resumed.initialize(ARGS, ids, lens, tg, st, **kw)
    try:
        for n in names:     # the resumed context starts from the saved values (no optimizer step yet)
            np.testing.assert_array_equal(resumed._trainer.get(n, 0, saved[n].shape), saved[n])
    finally:
        resumed._trainer.close()


@pytest.mark.gpu
def test_reference_calls_adain_and_pretrained_emb_disc_all():
    """args.adain trains through the reference's calls (initialize / add_loss / add_optimizer) like
    TacotronTrainer(style='adain').step_text, bit for bit; args.pretrained_emb_disc_all builds the
    training forward on the reference embeddings themselves, and its add_loss fails like the
    reference's without the unpaired towers (tacotron.py:808-811 index tower_refnet_out_up_emt)."""
    from oracle import train_ref as TRN
    from tt2.train import TacotronTrainer
    hp = _hp()
    W = init_tacotron_weights(hp, seed=5339, style="adain")
    ids, lens, re, rs, _, st, m = _batch(hp, T_ref=40)
    _, _, tg, _ = train_batch(ids.shape[0], ids.shape[1], 6, memory_width(hp, style="adain"), seed=32)
    B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
    args = types.SimpleNamespace(**dict(vars(ARGS), adain=True))
    model = _model(hp, W)
    got = []
    for step in range(2):
        model.initialize(args, ids, lens, tg, st, is_training=True, ref_mel_emt=re, ref_mel_spk=rs, train_masks=m)
        got.append(model.add_loss())
        assert model.add_optimizer(step) == step + 1
    names = TRN.frontend_var_names(adain=True) + TRN.train_var_names() + TRN.postnet_var_names()
    params = {n: model._trainer.get(n, 0, np.asarray(W[n]).shape) for n in names}
    model._trainer.close()
    tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1], style="adain")
    try:
        for step in range(2):
            L = tr.step_text(ids, lens, re, rs, tg, st, m["prenet"], m["zoneout"], m["postnet"], m["enc_conv"],
                             m["enc_zoneout"])
            assert got[step] == L["loss"]
        for n in names:
            assert np.array_equal(params[n], tr.get(n, 0, params[n].shape)), n
        moved = [n for n in names if "refnet/" in n and not np.array_equal(params[n], np.asarray(W[n], np.float32))]
        assert len(moved) >= 8, moved   # both conv stacks, the GRU and the dense were updated
    finally:
        tr.close()
    # pretrained_emb_disc_all: forward on refnet_emt / refnet_spk's embeddings, add_loss as the reference's
    W2 = init_tacotron_weights(hp, seed=5339, style="embed")   # memory width 2U + 2 x 128 (tacotron.py:284-291)
    ids, lens, re, rs, tg, st, m = _batch(hp, T_ref=40)
    model = _model(hp, W2)
    model.initialize(types.SimpleNamespace(**dict(vars(ARGS), pretrained_emb_disc_all=True)), ids, lens, tg, st,
                     is_training=True, ref_mel_emt=re, ref_mel_spk=rs, train_masks=m)
    try:
        assert np.isfinite(model.tower_decoder_output[0]).all()
        assert model._trainer.cfg.use_gst == 0 and model._trainer.cfg.n_emt == 0
        with pytest.raises(IndexError):
            model.add_loss()
    finally:
        model._trainer.close()
