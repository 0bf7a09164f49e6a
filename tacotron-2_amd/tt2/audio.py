"""WAV writers of code/datasets/audio.py:12-20 (scipy.io.wavfile, int16 PCM, peak-normalised).

Only the writers the synthesis path calls are restated; STFT / Griffin-Lim / librosa feature
extraction are not on the path.
"""
import numpy as np


def save_wav(wav, path, sr):
    """audio.py:12-15: scale to 32767 / max(0.01, peak), write int16."""
    from scipy.io import wavfile
    wav = np.asarray(wav, np.float64) * (32767 / max(0.01, float(np.max(np.abs(wav))) if len(wav) else 0.01))
    wavfile.write(path, sr, wav.astype(np.int16))


def save_wavenet_wav(wav, path, sr, inv_preemphasize=False, k=0.97):
    """audio.py:17-20: same scaling (the fork leaves inv_preemphasis commented out)."""
    save_wav(wav, path, sr)
