"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference's GPU Griffin-Lim
(datasets/audio.py:131-176, 237-246, 283-296; GL_on_GPU=True, hparams.py:135) for checking
csrc/griffinlim.hip.  Never imported by the product (see oracle/__init__.py).

TF 1.x tf.contrib.signal semantics restated: stft = frame(win, hop, pad_end=False) · periodic
Hann(win) -> rfft(n_fft); inverse_stft = irfft(n_fft)[:win] · periodic Hann(win) -> overlap_and_add
(no window-sum normalisation).  librosa.filters.mel (Slaney scale, Slaney norm, librosa's
defaults) restated loop by loop, independently of tt2/audio.py.  Parity unpinned (TF and
librosa are absent).
"""
import math

import numpy as np


def mel_basis(sr, n_fft, n_mels, fmin, fmax):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm=1)."""
    def hz2mel(f):
        return f / (200.0 / 3) if f < 1000.0 else 15.0 + math.log(f / 1000.0) / (math.log(6.4) / 27.0)

    def mel2hz(m):
        return (200.0 / 3) * m if m < 15.0 else 1000.0 * math.exp((math.log(6.4) / 27.0) * (m - 15.0))

    lo, hi = hz2mel(fmin), hz2mel(fmax)
    pts = [mel2hz(lo + (hi - lo) * i / (n_mels + 1)) for i in range(n_mels + 2)]
    nf = n_fft // 2 + 1
    freqs = [i * (sr / 2.0) / (nf - 1) for i in range(nf)]
    W = np.zeros((n_mels, nf))
    for m in range(n_mels):
        a, c, b = pts[m], pts[m + 1], pts[m + 2]
        for k, f in enumerate(freqs):
            up = (f - a) / (c - a)
            down = (b - f) / (b - c)
            W[m, k] = max(0.0, min(up, down))
        W[m] *= 2.0 / (b - a)
    return W


def denormalize(D, hp):
    """audio.py:283-296 (symmetric / clipping variants)."""
    mx, mn = hp["max_abs_value"], hp["min_level_db"]
    if hp["symmetric_mels"]:
        x = np.clip(D, -mx, mx) if hp["allow_clipping"] else D
        return ((x + mx) * -mn / (2 * mx)) + mn
    x = np.clip(D, 0, mx) if hp["allow_clipping"] else D
    return (x * -mn / mx) + mn


def _hann(n):
    return 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / n)


def stft(y, win, hop, n_fft):
    nfr = 1 + (len(y) - win) // hop
    w = _hann(win)
    fr = np.stack([y[t * hop:t * hop + win] * w for t in range(nfr)])
    return np.fft.rfft(fr, n=n_fft, axis=-1)


def inverse_stft(X, win, hop, n_fft):
    fr = np.fft.irfft(X, n=n_fft, axis=-1)[:, :win] * _hann(win)
    T = X.shape[0]
    y = np.zeros((T - 1) * hop + win)
    for t in range(T):
        y[t * hop:t * hop + win] += fr[t]
    return y


def griffin_lim(S, hp, iters):
    """_griffin_lim_tensorflow: zero initial phase, est / max(1e-8, |est|)."""
    win, hop, n_fft = hp["win_size"], hp["hop_size"], hp["n_fft"]
    Sc = S.astype(np.complex128)
    y = inverse_stft(Sc, win, hop, n_fft)
    for _ in range(iters):
        est = stft(y, win, hop, n_fft)
        ang = est / np.maximum(1e-8, np.abs(est))
        y = inverse_stft(Sc * ang, win, hop, n_fft)
    return y


def inv_spectrogram(spec, hp, is_mel, iters):
    """inv_{mel,linear}_spectrogram_tensorflow (audio.py:131-143) -> waveform (float64)."""
    D = denormalize(np.asarray(spec, np.float64), hp)
    S = np.power(10.0, (D + hp["ref_level_db"]) * 0.05) ** (1.0 / hp["magnitude_power"])
    if is_mel:
        ib = np.linalg.pinv(mel_basis(hp["sample_rate"], hp["n_fft"], hp["num_mels"], hp["fmin"],
                                      hp["fmax"]))
        S = np.maximum(1e-10, S @ ib.T)
    return griffin_lim(S ** hp["power"], hp, iters)


def audio_hp(hp):
    return dict(max_abs_value=hp.max_abs_value, min_level_db=hp.min_level_db,
                ref_level_db=hp.ref_level_db, symmetric_mels=hp.symmetric_mels,
                allow_clipping=hp.allow_clipping_in_normalization,
                magnitude_power=hp.magnitude_power, power=hp.power, win_size=hp.win_size,
                hop_size=hp.hop_size, n_fft=hp.n_fft, sample_rate=hp.sample_rate,
                num_mels=hp.num_mels, fmin=hp.fmin, fmax=hp.fmax)
