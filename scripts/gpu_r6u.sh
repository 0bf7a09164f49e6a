# round 6: persistent backward -- the product partials as tagged granules (no P flags, no drains)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -40; tail -30 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; tail -1 $O/tests.log
TT2_TB_STAMP=400 TT2_TB_STAMP_FILE=$O/tb400.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1 > $O/st.json 2> $O/st.err || { echo "stamp run failed"; tail -5 $O/st.err; exit 1; }
python scripts/tb_stamps.py $O/tb400.bin
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
for rep in 1 2; do
  for v in def launch; do
    L=""; [ $v = nt ] && L="TT2_LIB=$GRAFT_REPO_ROOT/tacotron-2_amd/libtt2_nt.so"; [ $v = launch ] && L="TT2_TR_PERSIST_BWD=0"
    env $L timeout -k 10 300 python -u bench.py $B --train-steps 3 > $O/ab_$v.json 2> $O/ab_$v.err || { echo "train bench failed for $v"; tail -5 $O/ab_$v.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]);t=d['train'];print('$v', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'))"
  done
done
TT2_TP_STAMP=400 TT2_TP_STAMP_FILE=$O/tp400.bin timeout -k 10 300 python -u bench.py $B --train-steps 1 > $O/tp.json 2> $O/tp.err || { echo "forward stamp run failed"; tail -5 $O/tp.err; exit 1; }
echo "== forward stamps"; python scripts/tp_stamps.py $O/tp400.bin
