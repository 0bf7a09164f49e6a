# FALL-free d W_loc: training parity suites (persist on and off), A/B of the train leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/train.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error|assert" $O/train.log | head -20; tail -30 $O/train.log; exit 1; }
tail -2 $O/train.log
TT2_TR_PERSIST=1 timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/train_p.log 2>&1 || { echo "train tests (persist) failed"; grep -E "FAILED|Error|assert" $O/train_p.log | head -20; tail -30 $O/train_p.log; exit 1; }
tail -2 $O/train_p.log
B="python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for m in "1 1" "1 0" "0 1"; do
  set -- $m
  TT2_TR_PERSIST=$1 TT2_TR_DWLOC_CUM=$2 timeout -k 10 300 $B > $O/bench_$1$2.json 2> $O/bench_$1$2.err || { echo "bench failed $m"; tail -5 $O/bench_$1$2.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$1$2.json').read().strip().splitlines()[-1]);t=d['train'];print('persist=$1 dwcum=$2', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('loss_first'), t.get('grad_norm'))"
done
