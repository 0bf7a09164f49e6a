# persistent-decoder GPU cycle: parity tests, then a short bench (tag = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pd}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "persistent or full_dims" > gpurun_out/pd_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -50 gpurun_out/pd_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/pd_tests_$TAG.log
mkdir -p gpurun_out; TT2_STAMP_STEP=500 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-wavenet > gpurun_out/pd_bench_$TAG.json 2> gpurun_out/pd_bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/pd_bench_$TAG.err; exit 1; }
cat gpurun_out/pd_bench_$TAG.json
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pd_bench2_$TAG.json 2> gpurun_out/pd_bench2_$TAG.err || { echo "bench2 failed"; tail -20 gpurun_out/pd_bench2_$TAG.err; exit 1; }
cat gpurun_out/pd_bench2_$TAG.json
