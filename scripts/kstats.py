"""Top kernels of a rocprofv3 --stats kernel_stats.csv: python scripts/kstats.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print("{:9.2f} ms {:7d} {:9.2f} us  {}".format(float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]),
                                                   float(r["AverageNs"]) / 1e3, r["Name"][:90]))
print("total {:.2f} ms".format(tot / 1e6))
