# round 6: training parity tests (incl. the one-work-group refnet GRU), kernel trace, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ah
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_train.py tests/test_train_options.py tests/test_train_outputs_per_step.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2 > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -5 $O/prof.err; exit 1; }
python scripts/train_step_kernels.py $O/prof/run_kernel_trace.csv 12
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $B > $O/ab.json 2> $O/ab.err || { echo "train bench failed"; tail -5 $O/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);t=d['train'];print(t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'), t.get('losses_last'))"
done
