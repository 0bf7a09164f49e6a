# persistent-decoder change: parity (decoder / emt / long horizon), then decoder + emt variant A/B vs lib_head.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "persistent or parity or longhorizon or emt" > gpurun_out/spill_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/spill_tests.log | head -20; tail -30 gpurun_out/spill_tests.log; exit 1; }
tail -1 gpurun_out/spill_tests.log
for rep in 1 2; do
  for L in tree lib_head.so lib_wl.so; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train > gpurun_out/sp.json 2> gpurun_out/sp.err || { echo "bench failed for $L"; tail -5 gpurun_out/sp.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/sp.json').read().strip().splitlines()[-1]); print('$L', d['value'], d['phases']['decode_us_per_step'], 'emt', d['variants']['emt_attn_multihead']['decode_us_per_step'])"
  done
done
