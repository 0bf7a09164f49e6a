"""Input-type predicates and mu-law companding of code/wavenet_vocoder/util.py:13-127 (plots /
librosa helpers omitted)."""
import numpy as np


def _assert_valid_input_type(s):
    assert s == 'mulaw-quantize' or s == 'mulaw' or s == 'raw'


def is_mulaw_quantize(s):
    _assert_valid_input_type(s)
    return s == 'mulaw-quantize'


def is_mulaw(s):
    _assert_valid_input_type(s)
    return s == 'mulaw'


def is_raw(s):
    _assert_valid_input_type(s)
    return s == 'raw'


def is_scalar_input(s):
    return is_raw(s) or is_mulaw(s)


# Mu-law companding (util.py:29-127; nnmnkwii's generic.py restated).  The reference hard-codes
# mu = 255 inside every function whatever the argument says, and so do these.
def mulaw(x, mu=256):
    mu = 255
    x = np.asarray(x, np.float64)
    return np.sign(x) * np.log1p(mu * np.abs(x)) / np.log1p(mu)


def inv_mulaw(y, mu=256):
    mu = 255
    y = np.asarray(y, np.float64)
    return np.sign(y) * (1.0 / mu) * ((1.0 + mu) ** np.abs(y) - 1.0)


def mulaw_quantize(x, mu=256):
    mu = 255
    return ((mulaw(x, mu) + 1) / 2 * mu).astype(np.int64)


def inv_mulaw_quantize(y, mu=256):
    mu = 255
    return inv_mulaw(2 * np.asarray(y, np.float64) / mu - 1, mu)
