# kernel-trace only (tag = $1), decoder bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-tr}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-wavenet > gpurun_out/trace_$TAG.json 2>/dev/null
echo rc=$?
head -20 gpurun_out/trace_$TAG/run_kernel_stats.csv | cut -d, -f1-4
