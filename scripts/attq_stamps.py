"""Summarise k_tr_att_bwd_q stage stamps (TT2_ATTQ_STAMP=<step>, TT2_ATTQ_STAMP_FILE=<path>: int64
[B][4][16] s_memrealtime at 100 MHz): per stage, median / max over work-groups in us from each
work-group's own start, and the spread of the work-group starts."""
import sys

import numpy as np

NAMES = ["start", "staged", "d cum own", "s", "d align", "tanh bwd", "df mfma", "end"]
s = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 16)
s = s[s[:, 0] != 0]
r = (s - s[:, :1]) * 0.01
print("work-groups", len(s), "start spread us", (s[:, 0].max() - s[:, 0].min()) * 0.01)
for i, n in enumerate(NAMES):
    v = r[:, i]
    print("{:2d} {:12s} median {:7.2f}  max {:7.2f}".format(i, n, np.median(v), v.max()))
