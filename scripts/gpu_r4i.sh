# fused training products with prefetched epilogue operands: training tests, step A/B, kernel trace
# and TCC / FETCH counters of the training leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4i
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_gpu_train_api.py tests/test_train_options.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r4i/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4i/tests.log | head -20; tail -30 gpurun_out/r4i/tests.log; exit 1; }
tail -1 gpurun_out/r4i/tests.log
ARGS="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for rep in 1 2; do
  for F in 1 0; do
    TT2_TR_FUSED=$F timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4i/b$F.json 2> gpurun_out/r4i/b$F.err || { echo "bench failed"; tail -5 gpurun_out/r4i/b$F.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4i/b$F.json').read().strip().splitlines()[-1]); print('fused=$F', d['train']['ms_per_step'], d['phases']['decode_us_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r4i/prof.json 2>/dev/null && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r4i/tcc -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4i/fetch -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2>&1
echo rc=$?
