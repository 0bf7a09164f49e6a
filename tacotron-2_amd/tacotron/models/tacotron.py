"""Tacotron (code/tacotron/models/tacotron.py:25-680), synthesis path on MI355X.

``Tacotron.initialize`` keeps the reference's signature and argument validation but runs eagerly:
instead of building a TF graph it executes encoder → decoder loop → Postnet through libtt2.so and
stores numpy arrays in the reference's ``tower_*`` attributes (one list entry per tower).

Training keeps the reference's three calls (tacotron/train.py:104-139 builds them once and runs
them every step; here each call does its part of the step eagerly):
``initialize(..., is_training=True)`` runs the whole teacher-forced forward + backward (encoder,
both reference encoders + GST, decoder, Postnet; training-mode batch norm, dropout and zoneout)
on ``tt2.train.TacotronTrainer``, ``add_loss()`` exposes the losses under the reference's names,
``add_optimizer(global_step)`` runs the tower mean (RCCL, one process per tower), clip + Adam and
the moving-statistics update.
"""
import os

import numpy as np

from tt2.engine import TacotronEngine
from tt2.weights import init_tacotron_weights


def split_func(x, split_pos):
    """tacotron.py:16-23: un-concatenate the time-axis-packed multi-tower batch."""
    rst = []
    start = 0
    for i in range(split_pos.shape[0]):
        rst.append(x[:, start:start + split_pos[i]])
        start += split_pos[i]
    return rst


def split_towers(hp, inputs, input_lengths, split_infos, ref_mel_emt, ref_mel_spk, mel_targets):
    """Per-tower inputs exactly as the reference packs them (tacotron.py:83-138,
    tacotron_emt_attn.py:81-137): split_func on the time-axis-packed batch when
    tacotron_num_gpus > 1."""
    inputs = np.asarray(inputs, np.int32)
    input_lengths = np.asarray(input_lengths, np.int32).reshape(-1)
    ntow = hp.tacotron_num_gpus
    asf = lambda x: None if x is None else np.asarray(x, np.float32)  # noqa: E731
    if split_infos is not None and ntow > 1:
        split_infos = np.asarray(split_infos, np.int32)
        tower_inputs = split_func(inputs, split_infos[:, 0])
        tower_ref_emt = (split_func(asf(ref_mel_emt), split_infos[:, 5])
                         if ref_mel_emt is not None else [None] * ntow)
        tower_ref_spk = (split_func(asf(ref_mel_spk), split_infos[:, 6])
                         if ref_mel_spk is not None else [None] * ntow)
        tower_targets = (split_func(asf(mel_targets), split_infos[:, 1])
                         if mel_targets is not None else [None] * ntow)
        # tf.split(input_lengths, num_or_size_splits=tacotron_num_gpus) (tacotron.py:89): an
        # integer split, so the reference itself requires equal tower sizes
        if input_lengths.shape[0] % ntow:
            raise ValueError("input_lengths ({}) must split evenly over tacotron_num_gpus={} "
                             "(tacotron.py:89 tf.split)".format(input_lengths.shape[0], ntow))
        tower_lengths = np.split(input_lengths, ntow)
    else:
        tower_inputs, tower_lengths = [inputs], [input_lengths]
        tower_ref_emt, tower_ref_spk = [asf(ref_mel_emt)], [asf(ref_mel_spk)]
        tower_targets = [asf(mel_targets)]
    return tower_inputs, tower_lengths, tower_ref_emt, tower_ref_spk, tower_targets


def tower_masks(prenet_masks, i, row0, B):
    """prenet_masks covers every utterance of every tower, [max_iters, 2, ntow*B, P] in tower-major
    row order, or is a list with one [max_iters, 2, B, P] array per tower (None = device RNG)."""
    if prenet_masks is None:
        return None
    if isinstance(prenet_masks, (list, tuple)):
        return prenet_masks[i]
    return np.asarray(prenet_masks)[:, :, row0:row0 + B]


class Tacotron():
    """Tacotron-2 Feature prediction Model."""

    def __init__(self, hparams):
        self._hparams = hparams
        self._weights = None
        self._engine = None
        self.device = int(os.environ.get("LOCAL_RANK", "0")) if "TT2_DEVICE" not in os.environ \
            else int(os.environ["TT2_DEVICE"])
        self._trainer = None
        self._train_key = None

    # -- weights (replaces tf.train.Saver.restore, tacotron/synthesizer.py:93-94) -------------
    def load_weights(self, weights):
        """weights: dict {TF variable name: array} or path to a .npz with those keys."""
        if isinstance(weights, str):
            with np.load(weights, allow_pickle=False) as z:
                weights = {k: z[k] for k in z.files}
        self._weights = dict(weights)
        self._engine = None

    def load_checkpoint(self, checkpoint, scopes=None):
        """tf.train.Saver(var_list).restore(sess, checkpoint) without TensorFlow: read the TF
        tensor bundle ``checkpoint`` (a prefix, or a directory holding a ``checkpoint`` state file
        as tf.train.get_checkpoint_state reads it) with tt2.ckpt and overwrite the matching
        variables; ``scopes`` restricts the restore to names containing one of the substrings,
        like the reference's refnet restore (tacotron/train.py:284-285, 330-338:
        ``load_checkpoint('spk_disc/pretrained_model_emt_disc', scopes=['refnet_emt'])``).
        Returns the restored names."""
        from tt2 import ckpt
        prefix = ckpt.latest_checkpoint(checkpoint) if os.path.isdir(checkpoint) else checkpoint
        names = [n for n, _ in ckpt.list_variables(prefix) if n.startswith("Tacotron_model/")
                 and (scopes is None or any(sc in n for sc in scopes))]
        values = ckpt.read_checkpoint(prefix, set(names))
        if self._weights is None:
            self._weights = {}
        for n, v in values.items():
            if n in self._weights and self._weights[n].shape != v.shape:
                raise ValueError("checkpoint variable {} has shape {}, model expects {}".format(
                    n, v.shape, self._weights[n].shape))
            self._weights[n] = v.astype(np.float32)
        self._engine = None
        return sorted(values)

    def init_random_weights(self, seed=None, emt_only=False, style="gst"):
        """style: 'gst' | 'embed' (args.pretrained_emb_disc_all) | 'adain' (args.adain)."""
        hp = self._hparams
        self.load_weights(init_tacotron_weights(
            hp, hp.tacotron_random_seed if seed is None else seed, emt_only, style))

    def _get_engine(self, B, T_in, T_ref, max_iters, emt_only, constraint, style="gst"):
        if self._weights is None:
            raise RuntimeError("Tacotron weights not loaded: call load_weights() (checkpoint) or "
                               "init_random_weights()")
        e = self._engine
        if (e is None or not e.fits(B, T_in, T_ref, max_iters) or e.emt_only != emt_only
                or e.cfg.synthesis_constraint != int(constraint) or e.style != style):
            if e is not None:
                e.close()
            self._engine = None
            e = TacotronEngine(self._hparams, self._weights, max(B, 1), T_in, max(T_ref, 1),
                               max_iters, self.device, emt_only, constraint, style=style)
            self._engine = e
        return e

    def initialize(self, args, inputs, input_lengths, mel_targets=None, stop_token_targets=None,
                   linear_targets=None, targets_lengths=None, gta=False, global_step=None,
                   is_training=False, is_evaluating=False, split_infos=None, emt_labels=None,
                   spk_labels=None, emt_up_labels=None, spk_up_labels=None, spk_emb=None,
                   ref_mel_emt=None, ref_mel_spk=None, ref_mel_up_emt=None, ref_mel_up_spk=None,
                   use_emt_disc=False, use_spk_disc=False, use_intercross=False,
                   use_unpaired=False, n_emt=None, n_spk=None, synth=False,
                   prenet_masks=None, seed=0, train_masks=None, train_capacity=None,
                   precision="fp32"):
        """Same arguments as the reference (tacotron.py:31-35) plus the injected prenet dropout
        keep-masks ``prenet_masks`` [max_iters, 2, B_total, 256] over every tower's utterances in
        tower order, or a list with one [max_iters, 2, B, 256] array per tower (None = device RNG
        keyed by ``seed``).

        is_training=True: the training step's forward + backward (see the module docstring).
        ``train_masks`` = dict of injected keep bits of this process's tower (keys 'prenet',
        'zoneout', 'postnet', 'enc_conv', 'enc_zoneout' in the layouts TacotronTrainer takes;
        missing ones are drawn at the hparams' rates from a generator seeded by ``seed``);
        ``train_capacity`` = dict(max_T_in, max_T_out, max_T_ref) sizes the training context at
        the first call (default: that call's sizes); ``precision`` 'fp32' or 'bf16' (GEMM operands,
        configs[4])."""
        hp = self._hparams
        # argument validation, tacotron.py:48-71
        if mel_targets is None and stop_token_targets is not None:
            raise ValueError('no multi targets were provided but token_targets were given')
        if mel_targets is not None and stop_token_targets is None and not gta:
            raise ValueError('Mel targets are provided without corresponding token_targets')
        if not gta and hp.predict_linear == True and linear_targets is None and is_training:
            raise ValueError('Model is set to use post processing to predict linear spectrograms '
                             'in training but no linear targets given!')
        if gta and linear_targets is not None:
            raise ValueError('Linear spectrogram prediction is not supported in GTA mode!')
        if is_training and hp.mask_decoder and targets_lengths is None:
            raise RuntimeError('Model set to mask paddings but no targets lengths provided for the mask!')
        if is_training and is_evaluating:
            raise RuntimeError('Model can not be in training and evaluation modes at the same time!')
        if hp.tacotron_use_style_emb_disc and (n_emt == None or n_spk == None):
            raise ValueError('must specify number of emotions and number of speakers!')
        if use_unpaired and not (hp.tacotron_use_style_emb_disc):
            raise ValueError('trying to use unpaired ')
        if getattr(args, "nat_gan", False) and not (getattr(args, "unpaired", False)):
            print("USING NATURALNESS GAN WITHOUT UNPAIRED SAMPLES")
        if ref_mel_emt is None and ref_mel_spk is None:
            raise ValueError("must provide references")
        adain = getattr(args, "adain", False)
        emt_only = bool(getattr(args, "emt_only", False))
        if adain and (emt_only or getattr(args, "unpaired", False)):
            raise ValueError("must provide speaker reference to use AdaIn and Unpaired with AddIn "
                             "not implemented")
        if use_unpaired and not (getattr(args, "pretrained_emb_disc_all", False)):
            raise ValueError('must use unpaired with pretrained_emb_disc_all')
        # scope of the MI355X path
        if is_evaluating:
            raise NotImplementedError("the eval-loss graph (is_evaluating=True) is not built; "
                                      "evaluate by synthesis (gta=True) or a training step's losses")
        if use_unpaired:
            raise NotImplementedError("the unpaired decode (tacotron.py:389-461) is a training-graph "
                                      "branch (teacher-forced on mel_targets); synthesis never builds it")
        # style path (tacotron.py:236-308): AdaIN, the reference embeddings themselves
        # (pretrained_emb_disc_all, or hp.use_gst=False), or GST
        style = ("adain" if adain else
                 "embed" if getattr(args, "pretrained_emb_disc_all", False) else "gst")
        if ref_mel_emt is None or (ref_mel_spk is None and not emt_only):
            raise ValueError("must provide references")  # refnet_emt / refnet_spk inputs (:251-259)
        constraint = bool(getattr(args, "synth_constraint", False))
        if is_training:
            return self._initialize_training(
                inputs, input_lengths, mel_targets, stop_token_targets, targets_lengths, split_infos,
                ref_mel_emt, ref_mel_spk, emt_only, style, use_emt_disc or use_spk_disc or use_intercross,
                train_masks, train_capacity, precision, seed, n_emt, n_spk, emt_labels, spk_labels)

        tower_inputs, tower_lengths, tower_ref_emt, tower_ref_spk, tower_targets = split_towers(
            hp, inputs, input_lengths, split_infos, ref_mel_emt, ref_mel_spk, mel_targets)
        self.tower_decoder_output = []
        self.tower_alignments = []
        self.tower_stop_token_prediction = []
        self.tower_mel_outputs = []
        self.tower_encoder_outputs = []
        self.tower_style_embeddings = []
        self.tower_linear_outputs = []
        self.tower_inputs = tower_inputs
        self.tower_input_lengths = tower_lengths
        self.tower_mel_targets = [t for t in tower_targets if t is not None]
        self.tower_ref_mel_emt = tower_ref_emt
        self.tower_ref_mel_spk = tower_ref_spk
        max_iters = hp.max_iters
        row0 = 0  # first utterance of tower i in the global (tower-major) row order
        for i in range(len(tower_inputs)):
            ids = np.ascontiguousarray(tower_inputs[i].reshape(tower_lengths[i].shape[0], -1))
            B, T_in = ids.shape
            ref_e = tower_ref_emt[i].reshape(B, -1, hp.num_mels)
            ref_s = None if tower_ref_spk[i] is None else tower_ref_spk[i].reshape(B, -1, hp.num_mels)
            T_ref = max(ref_e.shape[1], ref_s.shape[1] if ref_s is not None else 0)
            tg = None
            if gta and tower_targets[i] is not None:
                # every target frame: the decode feeds targets[:, r-1::r] itself (helpers.py:78)
                tg = tower_targets[i].reshape(B, -1, hp.num_mels)
            eng = self._get_engine(B, T_in, T_ref, max_iters, emt_only, constraint, style)
            masks = tower_masks(prenet_masks, i, row0, B)
            row0 += B
            out = eng.synthesize(ids, tower_lengths[i], ref_e, ref_s, max_iters, masks, seed, tg)
            self.tower_decoder_output.append(out["decoder_output"])
            self.tower_alignments.append(out["alignments"])
            self.tower_stop_token_prediction.append(out["stop_token_prediction"])
            self.tower_mel_outputs.append(out["mel_outputs"])
            self.tower_encoder_outputs.append(out["encoder_outputs"])
            self.tower_style_embeddings.append(out["style"][:, None, :])
            if hp.predict_linear and not gta:  # post_condition (tacotron.py:214, 466-481)
                self.tower_linear_outputs.append(eng.linear_outputs(out["mel_outputs"]))
        self.all_vars = list(self._weights.keys())

    # -- training (tacotron.py:31-35 is_training=True, add_loss :683, add_optimizer :1002) ----------
    def _tower_index(self, ntow):
        """This process's tower: one process per GPU (torch.distributed), rank r = tower r; the
        reference's towers share one process and average on the CPU (tacotron.py:1194-1208).
        Each rank passes either the packed batch of every tower (split_infos) or its own."""
        if ntow == 1:
            return 0
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() != ntow:
            raise NotImplementedError("tacotron_num_gpus={} towers train as one process per GPU: launch "
                                      "{} ranks (torch.distributed) or set tacotron_num_gpus=1".format(ntow, ntow))
        return dist.get_rank()

    def _initialize_training(self, inputs, input_lengths, mel_targets, stop_token_targets, targets_lengths,
                             split_infos, ref_mel_emt, ref_mel_spk, emt_only, style, disc, train_masks,
                             train_capacity, precision, seed, n_emt=None, n_spk=None, emt_labels=None,
                             spk_labels=None):
        from tt2 import synthetic as S
        from tt2.train import TacotronTrainer
        hp = self._hparams
        if mel_targets is None or stop_token_targets is None:
            raise ValueError("training needs mel_targets and stop_token_targets")
        # style paths in training (tacotron.py:236-308): GST (or hp.use_gst = False), AdaIN, and the
        # reference embeddings themselves for pretrained_emb_disc_all (whose add_loss the reference
        # can only run with the unpaired towers, see add_loss)
        self._train_style = style
        # use_emt_disc / use_spk_disc / use_intercross are stored and never read by the reference
        # graph (tacotron.py:74-76): accepted and ignored alike
        n_emt, n_spk = (int(n_emt or 0), int(n_spk or 0)) if hp.tacotron_use_style_emb_disc else (0, 0)
        if n_emt and emt_labels is None or (n_spk and not emt_only and spk_labels is None):
            raise ValueError("the style-embedding classifiers (tacotron_use_style_emb_disc) need emt_labels "
                             "and spk_labels")
        if self._weights is None:
            raise RuntimeError("Tacotron weights not loaded: call load_weights() (checkpoint) or "
                               "init_random_weights()")
        tower_inputs, tower_lengths, tower_ref_emt, tower_ref_spk, tower_targets = split_towers(
            hp, inputs, input_lengths, split_infos, ref_mel_emt, ref_mel_spk, mel_targets)
        ntow = len(tower_inputs)
        rank = self._tower_index(hp.tacotron_num_gpus)
        # the time-axis-packed batch of every tower (split_infos), or this rank's own batch
        i = rank if ntow > 1 else 0
        B = tower_lengths[i].shape[0]
        ids = np.ascontiguousarray(tower_inputs[i].reshape(B, -1))
        T_in = ids.shape[1]
        ref_e = np.ascontiguousarray(tower_ref_emt[i].reshape(B, -1, hp.num_mels))
        ref_s = (ref_e if emt_only or tower_ref_spk[i] is None
                 else np.ascontiguousarray(tower_ref_spk[i].reshape(B, -1, hp.num_mels)))
        T_ref = ref_e.shape[1]
        tg = np.ascontiguousarray(tower_targets[i].reshape(B, -1, hp.num_mels))
        T_out = tg.shape[1]
        stop = np.asarray(stop_token_targets, np.float32)
        if split_infos is not None and ntow > 1:
            stop = split_func(stop, np.asarray(split_infos, np.int32)[:, 2])[i]
        stop = np.ascontiguousarray(stop.reshape(B, T_out))
        tlen = None
        if targets_lengths is not None:
            tlen = np.split(np.asarray(targets_lengths, np.int32).reshape(-1), ntow)[i]
        cap = dict(max_T_in=T_in, max_T_out=T_out, max_T_ref=T_ref)
        cap.update(train_capacity or {})
        n_emt, n_spk = (int(n_emt or 0), int(n_spk or 0)) if hp.tacotron_use_style_emb_disc else (0, 0)
        if style != "gst":  # the AdaIN / pretrained_emb_disc_all graphs build no Style_Emb_Disc (:485-495)
            n_emt = n_spk = 0
        key = (B, emt_only, precision, n_emt, n_spk, style)
        tr = self._trainer
        if tr is not None and (self._train_key != key or T_in > self._train_cap["max_T_in"]
                               or T_out > self._train_cap["max_T_out"] or T_ref > self._train_cap["max_T_ref"]):
            raise ValueError("training batch {} exceeds the training context sized at the first step {}: "
                             "pass train_capacity= with the largest sizes on the first call".format(
                                 dict(B=B, T_in=T_in, T_out=T_out, T_ref=T_ref), self._train_cap))
        if tr is None:
            tr = TacotronTrainer(hp, self._weights, B, cap["max_T_in"], cap["max_T_out"], self.device,
                                 emt_only=emt_only, precision=precision, postnet=True, frontend=True,
                                 max_T_ref=cap["max_T_ref"], tf_seed=seed, n_emt=n_emt, n_spk=n_spk, style=style)
            self._trainer, self._train_key, self._train_cap = tr, key, cap
            # the classifiers' variables are trained and saved like the rest (tf.train.Saver)
            for k, v in tr.style_disc_weights.items():
                self._weights.setdefault(k, np.asarray(v, np.float32))
            self._mask_rng = np.random.default_rng(seed)
        tr.set_step_inputs(targets_lengths=tlen)
        if n_emt or n_spk:  # Style_Emb_Disc targets (tf.one_hot of the labels, tacotron.py:813-814)
            el = np.split(np.asarray(emt_labels, np.int32).reshape(-1), ntow)[i]
            sl = None if emt_only else np.split(np.asarray(spk_labels, np.int32).reshape(-1), ntow)[i]
            tr.set_style_labels(el, sl)
        m = dict(train_masks or {})
        r = self._mask_rng
        sub = lambda: int(r.integers(1 << 31))  # noqa: E731  (one fresh stream per mask per step)
        P, H, U = hp.prenet_layers[0], hp.decoder_lstm_units, hp.encoder_lstm_units
        zr, dr = hp.tacotron_zoneout_rate, hp.tacotron_dropout_rate
        T_dec = T_out // hp.outputs_per_step  # decoder steps (r frames each)
        masks = dict(
            prenet=m.get("prenet") if "prenet" in m else S.prenet_masks(T_dec, B, P, seed=sub()),
            zoneout=m.get("zoneout") if "zoneout" in m else S.zoneout_masks(T_dec, B, H, zr, seed=sub()),
            postnet=m.get("postnet") if "postnet" in m else S.postnet_masks(
                hp.postnet_num_layers, B, T_out, hp.postnet_channels, dr, seed=sub()),
            enc_conv=m.get("enc_conv") if "enc_conv" in m else S.enc_conv_masks(
                hp.enc_conv_num_layers, B, T_in, hp.enc_conv_channels, dr, seed=sub()),
            enc_zoneout=m.get("enc_zoneout") if "enc_zoneout" in m else S.enc_zoneout_masks(
                T_in, B, U, zr, seed=sub()))
        tr.forward_backward_text(ids, tower_lengths[i], ref_e, ref_s, tg, stop, masks["prenet"],
                                 masks["zoneout"], masks["postnet"], masks["enc_conv"], masks["enc_zoneout"])
        fr, st, al = tr.outputs(T_in, T_out)
        self.ratio = tr.ratio if tr.ratio is not None else 1.0
        self.tower_decoder_output = [fr]
        self.tower_stop_token_prediction = [st]   # logits: StopProjection skips the sigmoid in training
        self.tower_alignments = [al]
        self.tower_mel_outputs = [tr.mel_outputs(T_out)]
        self.tower_inputs, self.tower_input_lengths = [ids], [tower_lengths[i]]
        self.tower_mel_targets, self.tower_stop_token_targets = [tg], [stop]
        self.tower_ref_mel_emt, self.tower_ref_mel_spk = [ref_e], [ref_s]
        self.tower_linear_outputs = []
        self.all_vars = list(self._weights.keys())
        self._losses = None

    def add_loss(self):
        """tacotron.py:683-1000 for this process's tower: before / after / stop-token /
        regularization losses, the style-embedding classifier and orthogonality losses of the step
        initialize(is_training=True) just ran (the unpaired / GAN losses are 0: those graphs are
        not built)."""
        tr = self._trainer
        if tr is None:
            raise RuntimeError("add_loss: call initialize(..., is_training=True) first")
        if getattr(self, "_train_style", "gst") == "embed":
            # tacotron.py:808-811: with pretrained_emb_disc_all the loss reads the unpaired towers'
            # reference embeddings (tower_refnet_out_up_emt[i]), appended only when use_unpaired
            # (:603-607); without them the reference's add_loss fails indexing the empty list, and the
            # unpaired decode itself is out of scope here
            raise IndexError("list index out of range: pretrained_emb_disc_all's add_loss needs the unpaired "
                             "towers (tacotron.py:808-811), which this build does not construct")
        L = tr.losses()
        self._losses = L
        self.before_loss, self.after_loss = L["before"], L["after"]
        self.stop_token_loss, self.regularization_loss = L["stop_token"], L["regularization"]
        self.linear_loss = 0.0
        for n in ("style_emb_loss_up_emt", "style_emb_loss_up_spk", "style_emb_loss_mel_out_up_emt",
                  "style_emb_loss_mel_out_up_spk", "g_loss_p", "g_loss_up"):
            setattr(self, n, 0.0)
            setattr(self, "tower_" + n, [0.0])
        for n in ("style_emb_loss_emt", "style_emb_loss_spk", "style_emb_orthog_loss"):
            setattr(self, n, L[n])
            setattr(self, "tower_" + n, [L[n]])
        self.loss = L["loss"]
        self.loss_no_mo_up = L["loss"]
        self.tower_before_loss, self.tower_after_loss = [self.before_loss], [self.after_loss]
        self.tower_stop_token_loss = [self.stop_token_loss]
        self.tower_regularization_loss = [self.regularization_loss]
        self.tower_linear_loss = [0.0]
        self.tower_loss = [self.loss]
        return self.loss

    def add_optimizer(self, global_step=None):
        """tacotron.py:1002-1109: tower mean of the gradients (one RCCL all-reduce across the
        ranks), clip_by_global_norm(1.0), Adam at the decayed learning rate of ``global_step``
        (the value BEFORE this update, as TF reads the variable; None = the trainer's own count),
        then the batch-norm moving statistics (UPDATE_OPS) composed over the ranks.  Sets
        ``learning_rate``, ``optimize`` (the global step after the update) and ``grad_norm``."""
        tr = self._trainer
        if tr is None:
            raise RuntimeError("add_optimizer: call initialize(..., is_training=True) first")
        gs = tr.global_step if global_step is None else int(global_step)
        L = tr.optimizer_step(gs + 1)
        from tt2.train import learning_rate
        self.learning_rate = learning_rate(gs, self._hparams)
        self.optimize = tr.global_step
        self.grad_norm = L["grad_norm"]
        return self.optimize

    def trained_weights(self):
        """The trainer's current parameters as {TF variable name: array} (what tf.train.Saver
        would save), also made this model's weights for synthesis."""
        tr = self._trainer
        if tr is None:
            return dict(self._weights)
        from tt2._lib import TT2Error
        for n, v in list(self._weights.items()):
            try:
                self._weights[n] = tr.get(n, 0, np.asarray(v).shape)
            except TT2Error:  # not a variable of the training graph (e.g. the CBHG / emt heads)
                pass
        self._engine = None
        return dict(self._weights)
