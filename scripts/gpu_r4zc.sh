# bf16 values for the training step's per-step context / d align reads: training GPU tests,
# step A/B TT2_TR_VALUES16=1 vs 0 (same build), kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4zc
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_gpu_train_api.py tests/test_train_options.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r4zc/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error|^E " gpurun_out/r4zc/tests.log | head -20; tail -30 gpurun_out/r4zc/tests.log; exit 1; }
tail -1 gpurun_out/r4zc/tests.log
ARGS="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for rep in 1 2; do
  for v in 1 0; do
    TT2_TRAIN_BLAS=1 TT2_DUMMY=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4zc/b.json 2> gpurun_out/r4zc/b.err || { echo "bench failed"; tail -5 gpurun_out/r4zc/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4zc/b.json').read().strip().splitlines()[-1]); print('rep=$v', d['train']['ms_per_step'], d['train']['loss_last'], d['train']['grad_norm'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4zc/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r4zc/prof.json 2>/dev/null
echo rc=$?
