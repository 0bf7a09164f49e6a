"""Postnet-only driver for counter / trace passes: configs[1] shapes (B=32, T_out=1000, 512-ch
Postnet), random-init weights, N calls of tt2_postnet on fixed synthetic frames."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tacotron-2_amd"), ROOT]

from tt2.engine import TacotronEngine  # noqa: E402
from tt2.hparams import hparams  # noqa: E402
from tt2.weights import init_tacotron_weights  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B, T = 32, 1000
hp = hparams.copy()
hp.tacotron_num_gpus = 1
W = init_tacotron_weights(hp, seed=1)
eng = TacotronEngine(hp, W, B, 8, 64, T, 0, False, False)
frames = np.random.default_rng(0).uniform(-4, 4, (B, T, hp.num_mels)).astype(np.float32)
for i in range(n):
    t0 = time.time()
    eng.postnet(frames)
    print("postnet call", i, "%.3f ms (host, incl. copies)" % (1e3 * (time.time() - t0)), flush=True)
eng.close()
