# WaveNet-only GPU cycle: parity tests + generation bench (tag = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-w}
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "wavenet or mol" > gpurun_out/wn_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/wn_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/wn_tests_$TAG.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --t-out 50 --no-cpu-baseline --profile-iters 5 > gpurun_out/wn_bench_$TAG.json 2> gpurun_out/wn_bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/wn_bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/wn_bench_$TAG.json')); print(json.dumps(d['wavenet']))"
