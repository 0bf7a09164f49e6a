"""Persistent decoder step time at configs[1] shape (B = 32 x 201 chars, 1000 GTA steps so every launch
runs the full horizon), production kernel vs the arithmetic-free floor instance (TT2_PD_FLOOR=1, set
by the caller).  Prints us/step of the kernel (HIP events) for 3 launches."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tacotron-2_amd"))
from tt2.engine import TacotronEngine  # noqa: E402
from tt2.hparams import hparams  # noqa: E402
from tt2.synthetic import prenet_masks, tacotron_inputs  # noqa: E402
from tt2.weights import init_tacotron_weights  # noqa: E402

hp = hparams.copy()
B, T, TR, n = 32, 201, 400, 1000
hp.override_from_dict(dict(tacotron_num_gpus=1, max_iters=n))
W = init_tacotron_weights(hp, seed=hp.tacotron_random_seed)
ids, lens, re, rs = tacotron_inputs(B, T, TR, seed=1234, ragged=False)
tg = np.random.default_rng(1).uniform(-4, 4, (B, n, hp.num_mels)).astype(np.float32)
masks = prenet_masks(n, B, hp.prenet_layers[0], seed=1)
eng = TacotronEngine(hp, W, B, T, TR, n, 0)
res = []
for k in range(3):
    out = eng.synthesize(ids, lens, re, rs, n, masks, 0, tg)
    p, ms = eng.decoder_path()
    res.append(1e3 * ms / out["frames"].shape[1])
print("floor" if os.environ.get("TT2_PD_FLOOR") == "1" else "production", "persistent", p,
      "us/step", [round(v, 2) for v in res])
eng.close()
