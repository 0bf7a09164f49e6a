"""Summarise the persistent training forward's stage stamps (TT2_TP_STAMP=<step>,
TT2_TP_STAMP_FILE=<path>: int64 [256][32] s_memrealtime at 100 MHz): median / max over work-groups
of each stage in us from the step's earliest start."""
import sys

import numpy as np

NAMES = ["start", "L1 ctx waited", "L1 mfma", "L1 red", "H1 published", "H1 waited", "L2 mfma",
         "H2 published", "H2 waited", "hz1 part", "query", "qv", "energies", "hz2 part", "E taken",
         "softmax", "context", "CTX published", "prenet part"]
s = np.fromfile(sys.argv[1], dtype=np.int64).reshape(256, 32)
r = (s - s[:, 0].min()) * 0.01
for i, n in enumerate(NAMES):
    v = r[:, i][s[:, i] != 0]
    if len(v):
        print("{:2d} {:16s} median {:7.2f}  max {:7.2f}  min {:7.2f}".format(i, n, np.median(v), v.max(), v.min()))
