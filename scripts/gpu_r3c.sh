# training: row attention kernels (batched prefetch) parity + A/B vs tiles, register-direct GEMM A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train.py tests/test_train_options.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -2 gpurun_out/r3c_tests.log
for cfg in "TT2_TR_ATT_ROW=0" "TT2_TR_ATT_ROW=1" "TT2_GEMM_SKINNY=2" "TT2_TR_ATT_ROW=0 TT2_GEMM_SKINNY=2"; do
  env $cfg timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/r3c_t.json 2> gpurun_out/r3c_t.err || { echo "train bench failed $cfg"; tail -5 gpurun_out/r3c_t.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r3c_t.json').read().strip().splitlines()[-1]); print('$cfg', d['train']['ms_per_step'])"
done
TT2_GEMM_SKINNY=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/r3c_prof.json 2> gpurun_out/r3c_prof.err || { echo "prof failed"; tail -5 gpurun_out/r3c_prof.err; exit 1; }
head -16 gpurun_out/prof_r3c/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-110
