# parity (decoder + training), then decoder and training-step A/B: in-tree build vs lib_head.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "train or persistent or parity or longhorizon" > gpurun_out/combo_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/combo_tests.log | head -20; tail -30 gpurun_out/combo_tests.log; exit 1; }
tail -1 gpurun_out/combo_tests.log
for rep in 1 2; do
  for L in tree lib_head.so; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3 > gpurun_out/cb.json 2> gpurun_out/cb.err || { echo "bench failed for $L"; tail -5 gpurun_out/cb.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/cb.json').read().strip().splitlines()[-1]); print('$L', 'decode', d['phases']['decode_us_per_step'], 'train', d['train']['ms_per_step'], d['train']['loss_last'])"
  done
done
