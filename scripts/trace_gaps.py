"""Per-kernel in-chain durations and inter-kernel gaps of the decoder loop from a rocprofv3
--kernel-trace CSV (the decode loop = the longest run of k_prenet-started 7-kernel steps)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tt2::", "") for r in rows]
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
dur = defaultdict(list)
gap = defaultdict(list)
steps = []
for i, n in enumerate(names):
    if n.startswith("k_prenet"):
        steps.append(i)
for a, b in zip(steps, steps[1:]):
    if b - a != 7:
        continue
    for i in range(a, b):
        dur[names[i] + "@%d" % (i - a)].append((en[i] - st[i]) / 1000)
        gap[names[i] + "@%d" % (i - a)].append((st[i + 1] - en[i]) / 1000)
    steps_len = (st[b] - st[a]) / 1000
    dur["STEP"].append(steps_len)
for k in sorted(dur, key=lambda k: (k != "STEP", k.split("@")[-1])):
    v = sorted(dur[k])
    g = sorted(gap.get(k, [0]))
    print("%-24s n=%4d  dur med %7.2f us   gap-after med %5.2f us" % (k, len(v), v[len(v) // 2], g[len(g) // 2]))
