# register-direct skinny GEMM (TT2_GEMM_SKINNY=2): bf16 training parity, then train-step A/B + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TT2_GEMM_SKINNY=2 timeout -k 10 300 python -u -m pytest tests/test_train.py tests/test_train_options.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/rd_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rd_tests.log; exit 1; }
tail -2 gpurun_out/rd_tests.log
B="python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
for m in 0 2 0 2; do
  TT2_GEMM_SKINNY=$m timeout -k 10 200 $B > gpurun_out/rd_b$m.json 2> gpurun_out/rd_b$m.err || { echo "bench failed $m"; tail -5 gpurun_out/rd_b$m.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/rd_b$m.json').read().strip().splitlines()[-1]); print('mode $m', d['train']['ms_per_step'])"
done
TT2_GEMM_SKINNY=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rd -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/rd_prof.json 2> gpurun_out/rd_prof.err || { echo "prof failed"; tail -5 gpurun_out/rd_prof.err; exit 1; }
head -16 gpurun_out/prof_rd/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
