# round 6: persistent backward -- park behind the P1 poll; A/B of the nt cache policy on the step's
# streamed traffic (TT2_LIB=libtt2_nt.so, built with -DTB_NT=1) against the default build and the launches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -40; tail -30 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; tail -1 $O/tests.log
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
for lib in def nt; do
  L=""; [ $lib = nt ] && L="TT2_LIB=$GRAFT_REPO_ROOT/tacotron-2_amd/libtt2_nt.so"
  env $L TT2_TB_STAMP=400 TT2_TB_STAMP_FILE=$O/tb400_$lib.bin timeout -k 10 300 python -u bench.py $B --train-steps 1 > $O/st_$lib.json 2> $O/st_$lib.err || { echo "stamp run failed $lib"; tail -5 $O/st_$lib.err; exit 1; }
  echo "== stamps $lib"; python scripts/tb_stamps.py $O/tb400_$lib.bin
done
for rep in 1 2; do
  for v in def nt launch; do
    L=""; [ $v = nt ] && L="TT2_LIB=$GRAFT_REPO_ROOT/tacotron-2_amd/libtt2_nt.so"; [ $v = launch ] && L="TT2_TR_PERSIST_BWD=0"
    env $L timeout -k 10 300 python -u bench.py $B --train-steps 3 > $O/ab_$v.json 2> $O/ab_$v.err || { echo "train bench failed for $v"; tail -5 $O/ab_$v.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]);t=d['train'];print('$v', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'))"
  done
done
