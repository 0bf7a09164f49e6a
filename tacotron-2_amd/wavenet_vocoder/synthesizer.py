"""Synthesizer of code/wavenet_vocoder/synthesizer.py:13-131 on the MI355X path.

``load`` builds the eager ``WaveNet`` and restores weights: a TF tensor bundle holding the EMA
shadow variables the reference restores (``create_shadow_saver`` / ``load_averaged_model``,
wavenet_vocoder/train.py:67-86: ``<var>/ExponentialMovingAverage`` mapped onto ``<var>``), a
``.npz`` of TF-named arrays, or ``None`` for the seeded random initialisation.  ``synthesize``
keeps the reference's host-side batch preparation (audio lengths = mel frames x hop, clip to
T2_output_range, pad with its lower end to the longest mel, ``_interp`` to [0, 1]) and writes
``wavenet-audio-<basename>.wav`` per utterance (datasets/audio.py save_wavenet_wav).

Without local conditioning (``cin_channels <= 0``) the reference feeds ``synthesis_length = 100``
instead of the mels (synthesizer.py:51-53,75-78); here that runs ``tt2_wn_generate_unconditional``
(one row, or one per speaker id with global conditioning).  ``hparams.wavenet_synth_debug``
(synthesizer.py:56-58,83-95) swaps the mels for ``wavenet_debug_mels`` and teacher-forces the
generator with ``wavenet_debug_wavs`` (``.npy`` files, loaded without pickle).  Not reproduced (off
the hot path): the reconstructed-mel / upsampled-feature / waveform plots.
"""
import os

import numpy as np

from tt2.audio import save_wavenet_wav
from tt2.hparams import get_hop_size
from wavenet_vocoder.models import create_model


def _interp(feats, in_range):
    """wavenet_vocoder/feeder.py:426-428: rescale [-max, max] (or [0, max]) to [0, 1]."""
    return (feats - in_range[0]) / (in_range[1] - in_range[0])


#: synthesizer.py:78: samples generated per utterance without a local condition
SYNTHESIS_LENGTH = 100


def _pad_inputs(x, maxlen, _pad=0):
    return np.pad(x, [(0, maxlen - len(x)), (0, 0)], mode='constant', constant_values=_pad)


class Synthesizer:
    def load(self, checkpoint_path, hparams, model_name='WaveNet'):
        self._hparams = hparams
        self.synth_debug = bool(getattr(hparams, 'wavenet_synth_debug', False))
        self.model = create_model(model_name, hparams)
        if checkpoint_path is None:
            self.model.init_random_weights()
        elif str(checkpoint_path).endswith('.npz'):
            self.model.load_weights(checkpoint_path)
        else:
            self.model.init_random_weights()
            self.model.load_checkpoint(checkpoint_path)

    def synthesize(self, mel_spectrograms, speaker_ids, basenames, out_dir, log_dir, u_mix=None,
                   u_log=None, seed=0):
        """mel_spectrograms: list of [T_i, num_mels] arrays.  Returns the wav paths (or, with
        ``out_dir=None``, the trimmed waveforms)."""
        hp = self._hparams
        local_cond, global_cond = self._check_conditions()
        # synthesizer.py:56-58: debug mode swaps in the mels of the debug utterances
        if self.synth_debug:
            if len(hp.wavenet_debug_mels) != len(hp.wavenet_debug_wavs):
                raise ValueError('wavenet_debug_mels and wavenet_debug_wavs must pair up')
            mel_spectrograms = [np.load(f) for f in hp.wavenet_debug_mels]
        # synthesizer.py:71 (g = speaker ids [B, 1] int32) -> WaveNet.initialize's g
        n_utt = (len(mel_spectrograms) if mel_spectrograms is not None else
                 1 if speaker_ids is None else len(speaker_ids))
        g = None if (speaker_ids is None or not global_cond) else \
            np.asarray(speaker_ids, dtype=np.int32).reshape(n_utt, 1)
        if not local_cond:
            # synthesizer.py:75-78: no mel condition, synthesis_length = 100 samples per row; the
            # mels (when given) still set the trim lengths, as the reference computes them
            self.model.initialize(None, None, g, None, synthesis_length=SYNTHESIS_LENGTH, u_mix=u_mix,
                                  u_log=u_log, seed=seed)
            generated_wavs = [w for tower in self.model.tower_y_hat for w in tower]
            if mel_spectrograms is not None:
                hop = get_hop_size(hp)
                generated_wavs = [w[:len(m) * hop] for w, m in zip(generated_wavs, mel_spectrograms)]
            self.upsampled_features = [None] * len(generated_wavs)
            return self._save(generated_wavs, basenames, out_dir)
        mel_spectrograms = [np.asarray(m, np.float32) for m in mel_spectrograms]
        audio_lengths = [len(x) * get_hop_size(hp) for x in mel_spectrograms]
        maxlen = max([len(x) for x in mel_spectrograms])
        T2_output_range = (-hp.max_abs_value, hp.max_abs_value) if hp.symmetric_mels \
            else (0, hp.max_abs_value)
        if hp.clip_for_wavenet:
            mel_spectrograms = [np.clip(x, T2_output_range[0], T2_output_range[1])
                                for x in mel_spectrograms]
        c_batch = np.stack([_pad_inputs(x, maxlen, _pad=T2_output_range[0])
                            for x in mel_spectrograms]).astype(np.float32)
        if hp.normalize_for_wavenet:
            c_batch = _interp(c_batch, T2_output_range).astype(np.float32)
        test_inputs = None
        if self.synth_debug:
            # synthesizer.py:83-95: the debug wavs, zero-padded to the longest, teacher-force the
            # generator over the mels' samples
            test_wavs = [np.load(f).reshape(-1, 1) for f in hp.wavenet_debug_wavs]
            max_test_len = max(len(x) for x in test_wavs)
            test_inputs = np.stack([_pad_inputs(x, max_test_len) for x in test_wavs]).astype(np.float32)
            if max_test_len != maxlen * get_hop_size(hp):
                raise ValueError('debug wavs must hold len(mel) * hop_size samples ({} != {})'.format(
                    max_test_len, maxlen * get_hop_size(hp)))
            test_inputs = test_inputs.reshape(len(test_wavs), max_test_len)
        self.model.initialize(None, c_batch, g, None, test_inputs=test_inputs, u_mix=u_mix, u_log=u_log,
                              seed=seed)
        generated_wavs = [w for tower in self.model.tower_y_hat for w in tower]
        upsampled = [f for tower in self.model.tower_synth_upsampled_local_features for f in tower]
        generated_wavs = [w[:n] for w, n in zip(generated_wavs, audio_lengths)]
        self.upsampled_features = [f[:, :n] for f, n in zip(upsampled, audio_lengths)]
        return self._save(generated_wavs, basenames, out_dir)

    def _save(self, generated_wavs, basenames, out_dir):
        hp = self._hparams
        if out_dir is None:
            return generated_wavs
        os.makedirs(out_dir, exist_ok=True)
        audio_filenames = []
        for i, wav in enumerate(generated_wavs):
            audio_filename = os.path.join(out_dir, 'wavenet-audio-{}.wav'.format(basenames[i]))
            save_wavenet_wav(wav.copy(), audio_filename, sr=hp.sample_rate,
                             inv_preemphasize=hp.preemphasize, k=hp.preemphasis)
            audio_filenames.append(audio_filename)
        return audio_filenames

    def _check_conditions(self):
        return self._hparams.cin_channels > 0, self._hparams.gin_channels > 0
