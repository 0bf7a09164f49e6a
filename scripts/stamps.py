"""Summarise gpurun_out/pd_stamps.npy (TT2_STAMP_STEP stage stamps of k_decode_persist, 256 x 32
s_memrealtime values at 100 MHz) per stage: median / max over work-groups, proj vs other."""
import sys

import numpy as np

NAMES = {0: "start", 1: "A pre taken", 18: "A mfma", 19: "A red", 2: "H1 pub", 3: "after H1 pub", 4: "H1 wait",
         16: "B mfma", 17: "B red", 5: "H2 pub", 6: "prefetch", 7: "C start", 8: "energies", 9: "projh+RG1a",
         21: "softmax", 10: "CTX pub", 11: "CTX wait(proj)", 12: "PP put", 13: "RG2 tail0", 20: "PP take",
         14: "prenet", 15: "end"}
ORDER = [0, 1, 18, 19, 2, 3, 4, 16, 17, 5, 6, 7, 8, 9, 21, 10, 11, 12, 13, 20, 14, 15]
s = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pd_stamps.npy").astype(np.int64)
r = (s - s[:, 0].min()) * 0.01
g = np.arange(256)
for i in ORDER:
    line = f"{i:2d} {NAMES[i]:16s}"
    for k, m in (("all", g >= 0), ("proj", g < 176), ("other", g >= 176)):
        v = r[m, i][s[m, i] != 0]
        if len(v):
            line += f"  {k}: {np.median(v):6.2f} / {v.max():6.2f}"
    print(line)

# per-XCD view (slot 31 = HW_REG_XCC_ID of the work-group, slots 22..29 = wave w's context-load miss)
if s[:, 31].any() or (s[:, 31] == 0).all():
    xcc = s[:, 31]
    print("XCD of work-group g: g % 8 ->", [int(np.bincount(xcc[g % 8 == k]).argmax()) for k in range(8)])
    NAMES[30] = "14 + vmcnt(0)"
    for i in (13, 20, 14, 30, 15, 0, 1, 4):
        line = f"{i:2d} {NAMES[i]:16s}"
        for x in range(8):
            v = r[xcc == x, i][s[xcc == x, i] != 0]
            line += f" x{x}:{np.median(v):6.2f}" if len(v) else ""
        print(line)
    miss = (s[:, 22:30] != 0)
    print("context-load misses per XCD (waves):", [int(miss[xcc == x].sum()) for x in range(8)])
    tail = r[:, 15] - r[:, 14]
    print("L1 context-row tail (15 - 14) median per XCD:", [round(float(np.median(tail[xcc == x])), 2) for x in range(8)])
