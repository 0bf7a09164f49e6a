"""Tacotron_emt_attn (code/tacotron/models/tacotron_emt_attn.py:22-514), synthesis path on MI355X.

Same eager contract as ``Tacotron`` (tacotron.py here): ``initialize`` validates its arguments like
the reference and fills the ``tower_*`` attributes with numpy arrays computed by libtt2.so.  The
emotion attention type and reference-encoder head come from ``args.attn`` / ``args.emt_ref_gru``
(train.py:147-150); ``emt_labels`` feed the 'style_tokens' query.
"""
import numpy as np

from tt2.engine import TacotronEngine
from tt2.weights import init_tacotron_emt_weights

from .tacotron import Tacotron, split_towers, tower_masks


class Tacotron_emt_attn(Tacotron):
    """Tacotron-2 feature prediction with a per-step emotion attention."""

    def init_random_weights(self, seed=None, emt_only=False, attn="style_tokens",
                            emt_ref_gru="none", n_emt=4):
        hp = self._hparams
        self.load_weights(init_tacotron_emt_weights(
            hp, attn, emt_ref_gru, emt_only, n_emt,
            hp.tacotron_random_seed if seed is None else seed))

    def _get_emt_engine(self, B, T_in, T_ref, max_iters, emt_only, constraint, attn, ref_gru,
                        n_emt):
        if self._weights is None:
            raise RuntimeError("Tacotron weights not loaded: call load_weights() (checkpoint) or "
                               "init_random_weights()")
        e = self._engine
        key = (emt_only, int(constraint), attn, ref_gru, n_emt)
        if e is None or not e.fits(B, T_in, T_ref, max_iters) or getattr(e, "_emt_key", None) != key:
            if e is not None:
                e.close()
            self._engine = None
            e = TacotronEngine(self._hparams, self._weights, max(B, 1), T_in, max(T_ref, 1),
                               max_iters, self.device, emt_only, constraint, attn, ref_gru, n_emt)
            e._emt_key = key
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
        """Reference signature (tacotron_emt_attn.py:29-33) plus injected ``prenet_masks`` / ``seed``
        as in ``Tacotron.initialize``."""
        hp = self._hparams
        # argument validation, tacotron_emt_attn.py:46-79
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
        attn = getattr(args, "attn", None)
        if attn == 'style_tokens' and getattr(args, "unpaired", False):
            raise ValueError("attention style tokens and unpaired not implemented")
        if attn not in ("simple", "multihead", "style_tokens"):
            raise NotImplementedError("args.attn={!r}: the decoder cell then has no emotion "
                                      "attention and its LSTM input width differs from every "
                                      "built variant".format(attn))
        ref_gru = getattr(args, "emt_ref_gru", "none")
        emt_only = bool(getattr(args, "emt_only", False))
        if is_training or is_evaluating:
            raise NotImplementedError("training / eval-loss graphs of Tacotron_emt_attn are not "
                                      "built (synthesis only)")
        if use_unpaired:
            raise NotImplementedError("unpaired reference paths are not built")
        if attn != "style_tokens" and ref_mel_emt is None:
            raise ValueError("must provide references")
        if attn != "style_tokens" and not emt_only and ref_mel_spk is None:
            raise ValueError("must provide references")
        n_lab = 4 if n_emt is None else int(n_emt)   # synthesizer.py:45 builds with n_emt=4
        if attn == "style_tokens" and emt_labels is None:
            raise ValueError("style_tokens attention needs emt_labels")
        constraint = bool(getattr(args, "synth_constraint", False))

        tower_inputs, tower_lengths, tower_ref_emt, tower_ref_spk, tower_targets = split_towers(
            hp, inputs, input_lengths, split_infos, ref_mel_emt, ref_mel_spk, mel_targets)
        ntow = len(tower_inputs)
        tower_labels = (np.split(np.asarray(emt_labels, np.int32).reshape(-1), ntow)
                        if emt_labels is not None else [None] * ntow)   # tacotron_emt_attn.py:87
        self.tower_decoder_output = []
        self.tower_alignments = []
        self.tower_alignments_emt = []
        self.tower_stop_token_prediction = []
        self.tower_mel_outputs = []
        self.tower_encoder_outputs = []
        self.tower_inputs = tower_inputs
        self.tower_input_lengths = tower_lengths
        self.tower_mel_targets = [t for t in tower_targets if t is not None]
        self.tower_ref_mel_emt = tower_ref_emt
        self.tower_ref_mel_spk = tower_ref_spk
        max_iters = hp.max_iters
        row0 = 0
        for i in range(ntow):
            ids = np.ascontiguousarray(tower_inputs[i].reshape(tower_lengths[i].shape[0], -1))
            B, T_in = ids.shape
            use_refs = attn != "style_tokens"
            ref_e = tower_ref_emt[i].reshape(B, -1, hp.num_mels) if use_refs else None
            ref_s = (tower_ref_spk[i].reshape(B, -1, hp.num_mels)
                     if use_refs and not emt_only else None)
            T_ref = max([r.shape[1] for r in (ref_e, ref_s) if r is not None] or [1])
            tg = None
            if gta and tower_targets[i] is not None:
                # every target frame: the decode feeds targets[:, r-1::r] itself (helpers.py:78)
                tg = tower_targets[i].reshape(B, -1, hp.num_mels)
            eng = self._get_emt_engine(B, T_in, T_ref, max_iters, emt_only, constraint, attn,
                                       ref_gru, n_lab)
            if tower_labels[i] is not None:
                eng.set_emt_labels(tower_labels[i])
            masks = tower_masks(prenet_masks, i, row0, B)
            row0 += B
            out = eng.synthesize(ids, tower_lengths[i], ref_e, ref_s, max_iters, masks, seed, tg)
            self.tower_decoder_output.append(out["decoder_output"])
            self.tower_alignments.append(out["alignments"])
            self.tower_stop_token_prediction.append(out["stop_token_prediction"])
            self.tower_mel_outputs.append(out["mel_outputs"])
            self.tower_encoder_outputs.append(out["encoder_outputs"])
            if attn == "simple":   # alignment_history_emt, [B, T_v, steps] (:482-487)
                self.tower_alignments_emt.append(eng.emt_alignments()[:, 0])
        self.all_vars = list(self._weights.keys())
