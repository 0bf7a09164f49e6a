# training large products on the hand-written bf16 kernel (gemm_bf16_kc) instead of rocBLAS:
# training GPU tests, step A/B against the previous build (variants/lib_prev.so), kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4w
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_gpu_train_api.py tests/test_train_options.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r4w/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4w/tests.log | head -20; tail -30 gpurun_out/r4w/tests.log; exit 1; }
tail -1 gpurun_out/r4w/tests.log
ARGS="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for rep in 1 2; do
  for L in tree variants/lib_prev.so; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4w/b.json 2> gpurun_out/r4w/b.err || { echo "bench failed"; tail -5 gpurun_out/r4w/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4w/b.json').read().strip().splitlines()[-1]); print('$L', d['train']['ms_per_step'], d['train']['loss_last'], d['train']['grad_norm'])"
  done
done
unset TT2_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4w/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r4w/prof.json 2>/dev/null
echo rc=$?
