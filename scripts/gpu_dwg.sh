# attention backward with the in-kernel d W_loc accumulators: training suites, then the train leg A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/train.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error|assert" $O/train.log | head -20; tail -30 $O/train.log; exit 1; }
tail -2 $O/train.log
B="python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for q in 1 0; do
  TT2_TR_ATTQ=$q timeout -k 10 300 $B > $O/bench_q$q.json 2> $O/bench_q$q.err || { echo "bench failed q=$q"; tail -5 $O/bench_q$q.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_q$q.json').read().strip().splitlines()[-1]);t=d['train'];print('attq=$q', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('loss_first'), t.get('loss_last'), t.get('grad_norm'))"
done
