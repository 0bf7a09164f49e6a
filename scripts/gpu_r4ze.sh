# encoder convs: K-split layers on the 256 x 256 LDS-DMA kernel (partials + k_cx_reduce) vs the
# 128 x 128 kernel (TT2_CX_WIDE_SPLIT=0), K split 2 / 4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ze
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "encoder or full_dims or postnet" --timeout 200 --timeout-method thread > gpurun_out/r4ze/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r4ze/tests.log | head; tail -20 gpurun_out/r4ze/tests.log; exit 1; }
tail -1 gpurun_out/r4ze/tests.log
ARGS="--steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train"
for rep in 1 2; do
  for v in "1 4" "0 4"; do
    set -- $v
    TT2_CX_WIDE_SPLIT=$1 TT2_ENC_SPLITK=$2 timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4ze/b.json 2> gpurun_out/r4ze/b.err || { echo "bench failed"; tail -5 gpurun_out/r4ze/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4ze/b.json').read().strip().splitlines()[-1]); print('wide=$1 ks=$2', d['value'], d['phases'])"
  done
done
