# round 6: direct refnet conv2d backward (parity vs the im2col form and the oracle) and the
# forward's off-chain placement (TT2_TP_OC) A/B at configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6af
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_train.py -k "refnet_conv_backward or frontend" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -40; tail -30 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; tail -1 $O/tests.log
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for rep in 1 2; do
  for cfg in "0 0" "0 1" "1 1" "3 1"; do
    set -- $cfg
    TT2_TP_OC=$1 TT2_FE_CONV_DIRECT=$2 timeout -k 10 300 python -u bench.py $B > $O/ab.json 2> $O/ab.err || { echo "train bench failed"; tail -5 $O/ab.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);t=d['train'];print('oc=$1 direct=$2', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'), t.get('losses_last'))"
  done
done
