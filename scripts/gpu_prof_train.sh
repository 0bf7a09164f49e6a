# kernel trace of the configs[4] train leg (persistent forward on)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
TT2_TR_PERSIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2 > $O/prof.json 2> $O/prof.err || { echo "rocprof failed"; tail -5 $O/prof.err; exit 1; }
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", round(tot / 1e6, 2))
for r in rows[:40]:
    print("{:>9.2f} ms {:>7} calls {:>10.1f} us  {}".format(float(r["TotalDurationNs"]) / 1e6, r["Calls"], float(r["AverageNs"]) / 1e3, r["Name"][:90]))
PY
