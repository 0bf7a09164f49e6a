"""Summarise the persistent training backward's stage stamps (TT2_TB_STAMP=<step>,
TT2_TB_STAMP_FILE=<path>: int64 [256][32] s_memrealtime at 100 MHz): median / max over work-groups
of each stage in us from the step's earliest start (train_bwd_persist.hip TB_STAMP indices)."""
import sys

import numpy as np

NAMES = ["start", "ATT P1 waited", "dctx", "granules out", "E taken", "dq", "Q published",
         "step end", "CELL2 waited", "G2 published", "P2 published", "CELL1 waited",
         "G1 published", "P1 published", "PROD2 polled", "PROD2 loads", "PROD2 staged", "PROD2 mfma",
         "PROD1 polled", "PROD1 loads", "PROD1 staged", "PROD1 mfma", "CELL1 loads", "CELL1 cell",
         "prefetch issued", "off-chain G", "off-chain M + barrier"]
s = np.fromfile(sys.argv[1], dtype=np.int64).reshape(256, 32)
r = (s - s[:, 0][s[:, 0] != 0].min()) * 0.01
for i, n in enumerate(NAMES):
    v = r[:, i][s[:, i] != 0]
    if len(v):
        print("{:2d} {:26s} median {:7.2f}  max {:7.2f}  min {:7.2f}  n {}".format(i, n, np.median(v), v.max(), v.min(), len(v)))
