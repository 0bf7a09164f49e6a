# training: GPU train tests on the in-tree build, then the train leg of bench.py under each library (in-tree = "tree")
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/trab_tests.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error|assert" gpurun_out/trab_tests.log | head -20; tail -30 gpurun_out/trab_tests.log; exit 1; }
tail -1 gpurun_out/trab_tests.log
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3 > gpurun_out/trab.json 2> gpurun_out/trab.err || { echo "train bench failed for $L"; tail -5 gpurun_out/trab.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/trab.json').read().strip().splitlines()[-1]);t=d['train'];print('$L', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'))"
  done
done
