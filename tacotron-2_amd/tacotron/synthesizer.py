"""Synthesizer of code/tacotron/synthesizer.py:19-387 on the MI355X path.

``load`` builds the eager ``Tacotron`` (tacotron/models) and restores weights: a TF tensor bundle
(prefix or directory, read by tt2.ckpt), a ``.npz`` of TF-named arrays, or ``None`` for the
seeded random initialisation.  ``synthesize`` keeps the reference's arguments and file contract:
``filenames_to_inputs`` pads ids per tower and reference mels with -max_abs_value, the stop
tokens give each row's length (``get_output_lengths``), mels are trimmed and clipped to
T2_output_range and written as ``<out_dir>/mels/mel-<basename>_<basename_ref>.npy`` (float32,
[T, 80]); with a ``log_dir`` each mel is also vocoded by the GPU Griffin-Lim
(``tt2.audio.inv_mel_spectrogram``) into ``<log_dir>/wavs/wav-<basename>_<ref>.wav`` like the
reference.  Not reproduced (off the hot path): alignment/spectrogram plots, live playback
(``basenames=None`` returns the mels instead of playing them).  The reference returns an always-empty ``saved_mels_paths`` (it never appends,
synthesizer.py:221); here it lists the files written, so ``run_eval``'s map.txt gets its rows.
"""
import os

import numpy as np

from tacotron.models import create_model
from tacotron.utils.text import text_to_sequence


class Synthesizer:
    def load(self, args, checkpoint_path, hparams, gta=False, use_intercross=False, n_emt=4,
             n_spk=2):
        self.args = args
        model_name = 'Tacotron_emt_attn' if getattr(args, 'emt_attn', False) else 'Tacotron'
        self.model = create_model(model_name, hparams)
        init = dict(emt_only=bool(getattr(args, 'emt_only', False)))
        if model_name == 'Tacotron_emt_attn':  # its variables depend on args.attn / emt_ref_gru
            init.update(attn=getattr(args, 'attn', None), emt_ref_gru=getattr(args, 'emt_ref_gru', 'none'),
                        n_emt=n_emt)
        else:  # style path of the Tacotron model (tacotron.py:236-308)
            init.update(style='adain' if getattr(args, 'adain', False) else
                        'embed' if getattr(args, 'pretrained_emb_disc_all', False) else 'gst')
        if checkpoint_path is None:
            self.model.init_random_weights(**init)
        elif str(checkpoint_path).endswith('.npz'):
            self.model.load_weights(checkpoint_path)
        else:
            self.model.init_random_weights(**init)
            self.model.load_checkpoint(checkpoint_path)
        self.gta = gta
        self._hparams = hparams

    def synthesize(self, texts, basenames, out_dir, log_dir, mel_filenames, basenames_refs=None,
                   mel_ref_filenames_emt=None, mel_ref_filenames_spk=None, emb_only=False,
                   emt_labels_synth=None, spk_labels_synth=None, prenet_masks=None, seed=0):
        hparams = self._hparams
        T2_output_range = (-hparams.max_abs_value, hparams.max_abs_value) if hparams.symmetric_mels \
            else (0, hparams.max_abs_value)
        texts = list(texts)
        basenames = None if basenames is None else list(basenames)
        if basenames_refs is None and basenames is not None:
            basenames_refs = ['ref'] * len(basenames)
        (basenames, basenames_refs, input_seqs, input_lengths, split_infos, mel_ref_seqs_emt,
         mel_ref_seqs_spk, emt_labels_synth, spk_labels_synth) = filenames_to_inputs(
            hparams, texts, basenames, mel_filenames, basenames_refs, mel_ref_filenames_emt,
            mel_ref_filenames_spk, emt_labels_synth, spk_labels_synth)
        targets = None
        if self.gta:  # the reference's (commented-out) GTA feed, synthesizer.py:127-140
            np_targets = [_load_mel(f) for f in mel_filenames]
            ntow = hparams.tacotron_num_gpus
            per = len(np_targets) // ntow
            for i in range(ntow):
                t, tl = _prepare_targets(np_targets[per * i:per * (i + 1)], hparams.outputs_per_step,
                                         -hparams.max_abs_value if hparams.symmetric_mels else 0)
                targets = t if targets is None else np.concatenate((targets, t), axis=1)
                split_infos[i][1] = tl
        self.model.initialize(self.args, input_seqs, input_lengths, mel_targets=targets,
                              gta=self.gta, split_infos=split_infos,
                              ref_mel_emt=mel_ref_seqs_emt, ref_mel_spk=mel_ref_seqs_spk,
                              emt_labels=emt_labels_synth, spk_labels=spk_labels_synth, synth=True,
                              n_emt=4, n_spk=2, prenet_masks=prenet_masks, seed=seed)
        if emb_only:
            if not hasattr(self.model, 'tower_style_embeddings'):
                raise NotImplementedError('emb_only of Tacotron_emt_attn (refnet / context outputs, '
                                          'synthesizer.py:136-142) is not exposed')
            return (self.model.tower_style_embeddings[0], None, None, None, 1.0)
        # Linearize outputs (n_gpus -> 1D), synthesizer.py:164-167
        mels = [m for tower in self.model.tower_mel_outputs for m in tower]
        alignments = [a for tower in self.model.tower_alignments for a in tower]
        stop_tokens = [s for tower in self.model.tower_stop_token_prediction for s in tower]
        if not self.gta:
            target_lengths = get_output_lengths(stop_tokens)
        else:
            target_lengths = [len(_load_mel(f)) for f in mel_filenames]
        mels = [mel[:tl, :] for mel, tl in zip(mels, target_lengths)]
        assert len(mels) == len(texts)
        mels = [np.clip(m, T2_output_range[0], T2_output_range[1]) for m in mels]
        self.alignments = alignments
        self.target_lengths = target_lengths
        if basenames is None:
            return mels
        saved_mels_paths, speaker_ids = [], []
        os.makedirs(os.path.join(out_dir, 'mels'), exist_ok=True)
        for i, mel in enumerate(mels):
            if hparams.gin_channels > 0:
                raise RuntimeError('global conditioning speaker ids are not set on this path '
                                   '(tacotron/synthesizer.py:213-214)')
            speaker_ids.append('<no_g>')
            mel_filename = os.path.join(out_dir, 'mels', 'mel-{}_{}.npy'.format(basenames[i],
                                                                               basenames_refs[i]))
            np.save(mel_filename, mel.astype(np.float32), allow_pickle=False)
            saved_mels_paths.append(mel_filename)
            if log_dir is not None and len(mel):
                # mel -> wav through the GPU Griffin-Lim (GL_on_GPU, synthesizer.py:199-206),
                # 0.5 s of silence on both sides
                from tt2.audio import inv_mel_spectrogram, save_wav
                os.makedirs(os.path.join(log_dir, 'wavs'), exist_ok=True)
                wav = inv_mel_spectrogram(mel, hparams)
                pad = np.zeros(int(.5 * hparams.sample_rate))
                save_wav(np.concatenate([pad, wav, pad]),
                         os.path.join(log_dir, 'wavs/wav-{}_{}.wav'.format(basenames[i], basenames_refs[i])),
                         sr=hparams.sample_rate)
        return saved_mels_paths, speaker_ids


def filenames_to_inputs(hparams, texts, basenames, mel_filenames, basenames_refs=None,
                        mel_ref_filenames_emt=None, mel_ref_filenames_spk=None,
                        emt_labels_synth=None, spk_labels_synth=None):
    """synthesizer.py:296-371.  Reference mels may be paths or arrays."""
    pad = 0
    target_pad = -hparams.max_abs_value if hparams.symmetric_mels else 0
    cleaner_names = [x.strip() for x in hparams.cleaners.split(',')]
    if mel_ref_filenames_emt is None and mel_ref_filenames_spk is None:
        raise ValueError('must provide references')  # tacotron.py:66-67
    lists = [texts, basenames, basenames_refs, mel_filenames, mel_ref_filenames_emt,
             mel_ref_filenames_spk, emt_labels_synth, spk_labels_synth]
    lists = [None if l is None else list(l) for l in lists]
    (texts, basenames, basenames_refs, mel_filenames, mel_ref_filenames_emt,
     mel_ref_filenames_spk, emt_labels_synth, spk_labels_synth) = lists
    # repeat the last sample until the batch divides (synthesizer.py:305-321)
    while len(texts) % hparams.tacotron_synthesis_batch_size != 0:
        for l in lists:
            if l is not None:
                l.append(l[-1])
    assert 0 == len(texts) % hparams.tacotron_num_gpus
    seqs = [np.asarray(text_to_sequence(text, cleaner_names)) for text in texts]
    input_lengths = [len(seq) for seq in seqs]
    size_per_device = len(seqs) // hparams.tacotron_num_gpus
    np_refs_emt = [_load_mel(f) for f in mel_ref_filenames_emt] if mel_ref_filenames_emt is not None \
        else None
    np_refs_spk = [_load_mel(f) for f in mel_ref_filenames_spk] if mel_ref_filenames_spk is not None \
        else None
    input_seqs = mel_ref_seqs_emt = mel_ref_seqs_spk = None
    split_infos = []
    for i in range(hparams.tacotron_num_gpus):
        sl = slice(size_per_device * i, size_per_device * (i + 1))
        d_in, max_seq_len = _prepare_inputs(seqs[sl], pad)
        input_seqs = d_in if input_seqs is None else np.concatenate((input_seqs, d_in), axis=1)
        len_e = len_s = 0
        if np_refs_emt is not None:
            d_e, len_e = _prepare_targets(np_refs_emt[sl], hparams.outputs_per_step, target_pad)
            mel_ref_seqs_emt = d_e if mel_ref_seqs_emt is None else \
                np.concatenate((mel_ref_seqs_emt, d_e), axis=1)
        if np_refs_spk is not None:
            d_s, len_s = _prepare_targets(np_refs_spk[sl], hparams.outputs_per_step, target_pad)
            mel_ref_seqs_spk = d_s if mel_ref_seqs_spk is None else \
                np.concatenate((mel_ref_seqs_spk, d_s), axis=1)
        split_infos.append([max_seq_len, 0, 0, 0, 0, len_e, len_s])
    input_lengths = np.asarray(input_lengths, dtype=np.int32)
    spk_labels_synth = None if spk_labels_synth is None else np.asarray(spk_labels_synth, np.int32)
    emt_labels_synth = None if emt_labels_synth is None else np.asarray(emt_labels_synth, np.int32)
    split_infos = np.asarray(split_infos, dtype=np.int32)
    return (basenames, basenames_refs, input_seqs, input_lengths, split_infos, mel_ref_seqs_emt,
            mel_ref_seqs_spk, emt_labels_synth, spk_labels_synth)


def _load_mel(f):
    """mel-*.npy [T, num_mels] (np.save'd float32; never unpickled) or an array."""
    return np.load(f, allow_pickle=False) if isinstance(f, str) else np.asarray(f, np.float32)


def _round_up(x, multiple):
    remainder = x % multiple
    return x if remainder == 0 else x + multiple - remainder


def _prepare_inputs(inputs, pad):
    max_len = max([len(x) for x in inputs])
    return np.stack([_pad_input(x, max_len, pad) for x in inputs]), max_len


def _pad_input(x, length, pad):
    return np.pad(x, (0, length - x.shape[0]), mode='constant', constant_values=pad)


def _prepare_targets(targets, alignment, target_pad):
    max_len = max([len(t) for t in targets])
    data_len = _round_up(max_len, alignment)
    return np.stack([_pad_target(t, data_len, target_pad) for t in targets]), data_len


def _pad_target(t, length, target_pad):
    return np.pad(t, [(0, length - t.shape[0]), (0, 0)], mode='constant',
                  constant_values=target_pad)


def get_output_lengths(stop_tokens):
    """synthesizer.py:384-387: first index where round(stop) == 1, else the row length."""
    return [row.index(1) if 1 in row else len(row) for row in np.round(stop_tokens).tolist()]
