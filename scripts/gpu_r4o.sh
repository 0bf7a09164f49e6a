# Postnet over pre-split padded planes (conv_x3): parity tests, bench A/B against the im2col
# GEMM path (TT2_POSTNET_CX=0), kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "postnet or full_dims" --timeout 120 --timeout-method thread > gpurun_out/r4o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4o/tests.log | head -20; tail -30 gpurun_out/r4o/tests.log; exit 1; }
tail -1 gpurun_out/r4o/tests.log
ARGS="--steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train"
for rep in 1 2; do
  for cx in 11 01 10; do
    TT2_POSTNET_CX=${cx:0:1} TT2_CX_WIDE=${cx:1:1} timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4o/b.json 2> gpurun_out/r4o/b.err || { echo "bench failed"; tail -5 gpurun_out/r4o/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4o/b.json').read().strip().splitlines()[-1]); print('cx=$cx', d['value'], d['phases'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4o/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r4o/prof.json 2>/dev/null
echo rc=$?
