# text encoder on the planes path (split-K conv_x3 + width-1 projection): parity tests, encode A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4q
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "postnet or full_dims or encoder" --timeout 120 --timeout-method thread > gpurun_out/r4q/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4q/tests.log | head -20; tail -30 gpurun_out/r4q/tests.log; exit 1; }
tail -1 gpurun_out/r4q/tests.log
ARGS="--steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train"
for rep in 1 2; do
  for v in "1 4" "0 4" "1 2" "1 6"; do
    set -- $v
    TT2_ENC_CX=$1 TT2_ENC_SPLITK=$2 timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4q/b.json 2> gpurun_out/r4q/b.err || { echo "bench failed"; tail -5 gpurun_out/r4q/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4q/b.json').read().strip().splitlines()[-1]); print('cx,ks=$1,$2', d['value'], d['phases'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4q/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r4q/prof.json 2>/dev/null
echo rc=$?
