"""tt2 — MI355X-native Tacotron-2 decoder + WaveNet MoL vocoder synthesis (host side).

The compute path is libtt2.so (hand-written gfx950 HIP kernels behind the C ABI in
include/tt2.h); this package is the ctypes binding, hparams and weight key space.
"""
from .hparams import HParams, hparams, paper_hparams  # noqa: F401

__version__ = "0.1.0"
