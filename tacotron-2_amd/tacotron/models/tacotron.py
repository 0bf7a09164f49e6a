"""Tacotron (code/tacotron/models/tacotron.py:25-680), synthesis path on MI355X.

``Tacotron.initialize`` keeps the reference's signature and argument validation but runs eagerly:
instead of building a TF graph it executes encoder → decoder loop → Postnet through libtt2.so and
stores numpy arrays in the reference's ``tower_*`` attributes (one list entry per tower).
Training through this class (is_training=True) would also train the encoder, GST and reference
encoders, whose backward is not built; the decoder + Postnet training step is
``tt2.train.TacotronTrainer``.
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
                   prenet_masks=None, seed=0):
        """Same arguments as the reference (tacotron.py:31-35) plus the injected prenet dropout
        keep-masks ``prenet_masks`` [max_iters, 2, B_total, 256] over every tower's utterances in
        tower order, or a list with one [max_iters, 2, B, 256] array per tower (None = device RNG
        keyed by ``seed``)."""
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
        if is_training or is_evaluating:
            raise NotImplementedError("training / eval-loss graphs of the whole model are not built "
                                      "(no encoder/GST backward); the decoder + Postnet training "
                                      "step is tt2.train.TacotronTrainer")
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
                tg = tower_targets[i].reshape(B, -1, hp.num_mels)[:, hp.outputs_per_step - 1::hp.outputs_per_step]
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
