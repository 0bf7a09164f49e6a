# rocprofv3 kernel-trace stats of the full default bench (decoder + WaveNet + E2E + Griffin-Lim legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.bench.json 2>/dev/null
echo rc=$?
