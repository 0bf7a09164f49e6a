# training-step A/B: in-tree build vs lib_head.so (training GPU tests first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "train" > gpurun_out/trab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/trab_tests.log; exit 1; }
tail -1 gpurun_out/trab_tests.log
for rep in 1 2; do
  for L in tree lib_head.so; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3 > gpurun_out/trab.json 2> gpurun_out/trab.err || { echo "bench failed for $L"; tail -5 gpurun_out/trab.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/trab.json').read().strip().splitlines()[-1]); print('$L', 'train', d['train']['ms_per_step'], d['train']['loss_last'])"
  done
done
