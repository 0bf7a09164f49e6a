"""Audio helpers of code/datasets/audio.py on the MI355X path.

* WAV writers (audio.py:12-20): scipy.io.wavfile, int16 PCM, peak-normalised.
* ``inv_mel_spectrogram`` / ``inv_linear_spectrogram``: the reference's GPU Griffin-Lim
  (GL_on_GPU=True, audio.py:131-176) through ``tt2_gl_*`` (csrc/griffinlim.hip), followed by the
  host-side ``inv_preemphasis`` (scipy lfilter, audio.py:27-30) exactly where the reference applies
  it (tacotron/synthesizer.py:153-154).
* ``build_mel_basis``: librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) (audio.py:243-246) —
  librosa is not installed, so the Slaney-scale, Slaney-normalised filterbank (librosa's default,
  htk=False, norm=1) is restated here; its pseudo-inverse (audio.py:234) is computed once on the
  host in float64, like the reference's ``np.linalg.pinv``.
Feature extraction (melspectrogram / STFT of training audio) is not on the synthesis path.
"""
import ctypes

import numpy as np


def save_wav(wav, path, sr):
    """audio.py:12-15: scale to 32767 / max(0.01, peak), write int16."""
    from scipy.io import wavfile
    wav = np.asarray(wav, np.float64) * (32767 / max(0.01, float(np.max(np.abs(wav))) if len(wav) else 0.01))
    wavfile.write(path, sr, wav.astype(np.int16))


def save_wavenet_wav(wav, path, sr, inv_preemphasize=False, k=0.97):
    """audio.py:17-20: same scaling (the fork leaves inv_preemphasis commented out)."""
    save_wav(wav, path, sr)


def inv_preemphasis(wav, k, inv_preemphasize=True):
    """audio.py:27-30: scipy.signal.lfilter([1], [1, -k], wav)."""
    if inv_preemphasize:
        from scipy import signal
        return signal.lfilter([1], [1, -k], wav)
    return wav


def _hz_to_mel(f):
    """librosa.hz_to_mel(htk=False): linear below 1 kHz (200/3 Hz per mel), log above."""
    f = np.asarray(f, np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep,
                    f / f_sp)


def _mel_to_hz(m):
    m = np.asarray(m, np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def build_mel_basis(hp):
    """librosa.filters.mel(hp.sample_rate, hp.n_fft, n_mels=hp.num_mels, fmin=hp.fmin,
    fmax=hp.fmax) -> [num_mels, n_fft/2+1] float64 (audio.py:243-246)."""
    assert hp.fmax <= hp.sample_rate // 2
    n_freq = 1 + hp.n_fft // 2
    fftfreqs = np.linspace(0, float(hp.sample_rate) / 2, n_freq)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(hp.fmin), _hz_to_mel(hp.fmax), hp.num_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    weights = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:hp.num_mels + 2] - mel_f[:hp.num_mels])
    return weights * enorm[:, None]


def gl_config(hp):
    from . import _lib
    lib = _lib.load_library()
    cfg = _lib.GlConfig()
    lib.tt2_gl_default_config(ctypes.byref(cfg))
    from .hparams import get_hop_size
    cfg.n_fft, cfg.hop_size = hp.n_fft, get_hop_size(hp)
    cfg.win_size = hp.win_size if hp.win_size is not None else hp.n_fft
    cfg.num_mels = hp.num_mels
    cfg.magnitude_power, cfg.power = hp.magnitude_power, hp.power
    cfg.ref_level_db, cfg.min_level_db = hp.ref_level_db, hp.min_level_db
    cfg.max_abs_value = hp.max_abs_value
    cfg.symmetric_mels = int(bool(hp.symmetric_mels))
    cfg.allow_clipping_in_normalization = int(bool(hp.allow_clipping_in_normalization))
    cfg.griffin_lim_iters = hp.griffin_lim_iters
    if not hp.signal_normalization:
        raise NotImplementedError("signal_normalization=False is not on the MI355X path")
    return cfg


class GriffinLim(object):
    """One tt2_gl_ctx (device) with the pinv(mel_basis) of ``hp`` uploaded."""

    def __init__(self, hp, device=0):
        from . import _lib
        self.lib = _lib.load_library()
        self.hp = hp
        self.cfg = gl_config(hp)
        h = ctypes.c_void_p()
        _lib.check(self.lib.tt2_gl_create(ctypes.byref(self.cfg), device, ctypes.byref(h)))
        self.h = h
        ib = np.ascontiguousarray(np.linalg.pinv(build_mel_basis(hp)), np.float32)  # [F, M]
        _lib.check(self.lib.tt2_gl_set_inv_mel_basis(self.h, _lib.ptr(ib)))

    def close(self):
        if getattr(self, "h", None):
            self.lib.tt2_gl_destroy(self.h)
            self.h = None

    __del__ = close

    def synthesize(self, spec, is_mel=True, iters=-1):
        """spec [T, num_mels] (mel) or [T, n_fft/2+1] (linear), normalised -> wav
        [(T-1)*hop + win] float32 (no inverse pre-emphasis)."""
        from . import _lib
        spec = np.ascontiguousarray(spec, np.float32)
        T = spec.shape[0]
        wav = np.zeros(((T - 1) * self.cfg.hop_size + self.cfg.win_size,), np.float32)
        _lib.check(self.lib.tt2_gl_synthesize(self.h, _lib.ptr(spec), T, int(bool(is_mel)), iters,
                                             _lib.ptr(wav)))
        return wav


_GL = {}


def _gl(hp):
    import os
    key = (hp.n_fft, hp.hop_size, hp.win_size, hp.num_mels, hp.sample_rate, hp.fmin, hp.fmax,
           hp.magnitude_power, hp.power, hp.griffin_lim_iters, hp.max_abs_value, hp.symmetric_mels)
    if key not in _GL:
        _GL[key] = GriffinLim(hp, int(os.environ.get("TT2_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    return _GL[key]


def inv_mel_spectrogram(mel_spectrogram, hparams):
    """Mel [T, num_mels] (as the Tacotron emits it) -> waveform, via the GPU Griffin-Lim of
    inv_mel_spectrogram_tensorflow + host inv_preemphasis (tacotron/synthesizer.py:153-154)."""
    wav = _gl(hparams).synthesize(mel_spectrogram, True)
    return inv_preemphasis(wav, hparams.preemphasis, hparams.preemphasize)


def inv_linear_spectrogram(linear_spectrogram, hparams):
    """Linear [T, n_fft/2+1] -> waveform (inv_linear_spectrogram_tensorflow + inv_preemphasis)."""
    wav = _gl(hparams).synthesize(linear_spectrogram, False)
    return inv_preemphasis(wav, hparams.preemphasis, hparams.preemphasize)
