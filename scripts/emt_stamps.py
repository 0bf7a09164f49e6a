"""Stage stamps of the Tacotron_emt_attn persistent decode (k_decode_persist<true>) at B = 32,
T_ref 400, step TT2_STAMP_STEP (default 300): medians per role (emotion rows g >= 240, emotion
query/dense blocks, the rest)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tacotron-2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
os.environ.setdefault("TT2_STAMP_STEP", "300")
from _common import full_hparams, prenet_masks, tacotron_inputs  # noqa: E402
from tt2 import _lib  # noqa: E402
from tt2.engine import TacotronEngine  # noqa: E402
from tt2.weights import init_tacotron_emt_weights  # noqa: E402

hp = full_hparams()
B, T, TR, n = 32, 201, 400, 600
W = init_tacotron_emt_weights(hp, "multihead", "gru", seed=5339)
ids, lens, re, rs = tacotron_inputs(B, T, TR, seed=7)
masks = prenet_masks(n, B, hp.prenet_layers[0], seed=7)
eng = TacotronEngine(hp, W, B, T, TR, n, 0, False, False, "multihead", "gru", 4)
eng.synthesize(ids, lens, re, rs, n, masks)
print("persistent", eng.decoder_path())
st = (ctypes.c_longlong * 8192)()
_lib.check(eng.lib.tt2_debug_pd_stamps(eng.h, st))
s = np.array(st[:], dtype=np.int64).reshape(256, 32)
r = (s - s[:, 0][s[:, 0] > 0].min()) * 0.01
g = np.arange(256)
isq = np.array([(x < 240) and (x % 30 >= 22) for x in g])
roles = {"emt": g >= 240, "q": isq, "proj": (g < 240) & ~isq}
for i in range(32):
    line = "%2d" % i
    any_ = False
    for k, m in roles.items():
        v = r[m, i][s[m, i] != 0]
        if len(v):
            any_ = True
            line += "  %s: %6.2f / %6.2f" % (k, np.median(v), v.max())
    if any_:
        print(line)
eng.close()
