# 256-thread attention energy kernels: training parity, A/B (TT2_TR_E2), kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train.py tests/test_train_options.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/e2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/e2_tests.log; exit 1; }
tail -2 gpurun_out/e2_tests.log
for cfg in "TT2_TR_E2=1" "TT2_TR_E2=0" "TT2_TR_E2=1"; do
  env $cfg timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/e2_t.json 2> gpurun_out/e2_t.err || { echo "train bench failed"; tail -5 gpurun_out/e2_t.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/e2_t.json').read().strip().splitlines()[-1]); print('$cfg train ms', d['train']['ms_per_step'], d['train']['loss_first'], d['train']['grad_norm'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/e2_prof.json 2> gpurun_out/e2_prof.err || { echo "prof failed"; tail -5 gpurun_out/e2_prof.err; exit 1; }
grep -E "att_|tr_ctx" gpurun_out/prof_e2/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-110
