# round 6: outputs_per_step r > 1 in the training step; training regressions and the configs[4] step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ac
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_train_outputs_per_step.py > $O/r.log 2>&1 || { echo "r tests failed"; grep -E "FAILED|Error|assert" $O/r.log | head -40; tail -40 $O/r.log; exit 1; }
grep -cE "PASSED" $O/r.log; tail -1 $O/r.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -40; tail -30 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; tail -1 $O/tests.log
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $B --train-steps 3 > $O/ab.json 2> $O/ab.err || { echo "train bench failed"; tail -5 $O/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);t=d['train'];print(t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'), t.get('losses_last'))"
done
