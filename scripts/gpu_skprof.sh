# round 3: per-kernel times of the training leg, skinny GEMM off / on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --no-variants"
for v in 0 1; do
TT2_GEMM_SKINNY=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/skp$v -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/skp$v.json 2> gpurun_out/skp$v.err || exit 1
done
python3 - <<'PY'
import csv
for v in (0, 1):
    rows = list(csv.DictReader(open("gpurun_out/skp%d/run_kernel_stats.csv" % v)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print("== skinny", v)
    for r in rows[:14]:
        print("%-60s %7s %10.2f us %8.1f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
