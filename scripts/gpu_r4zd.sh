# BiLSTM encoder: input projections prefetched before the h hand-off; sentinel poll on/off; A/B
# against the previous build (variants/lib_prev.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4zd
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "encoder or full_dims or gta_full" --timeout 200 --timeout-method thread > gpurun_out/r4zd/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r4zd/tests.log | head; tail -20 gpurun_out/r4zd/tests.log; exit 1; }
tail -1 gpurun_out/r4zd/tests.log
ARGS="--steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train"
for rep in 1 2; do
  for v in "tree 1" "tree 0" "prev 1"; do
    set -- $v
    if [ "$1" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/variants/lib_prev.so; fi
    TT2_ENC_SENTINEL=$2 timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4zd/b.json 2> gpurun_out/r4zd/b.err || { echo "bench failed"; tail -5 gpurun_out/r4zd/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4zd/b.json').read().strip().splitlines()[-1]); print('$1 sent=$2', d['value'], d['phases'])"
  done
done
