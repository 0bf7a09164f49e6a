# persistent training forward (thread-per-position energies) + bf16 d-align reads: small case,
# stamps, A/B of the train leg, training parity suites, kernel trace of the persistent train leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/dbg_tp_small.py 5 7 3 > $O/small.log 2>&1 || { echo "small failed"; tail -5 $O/small.log; exit 1; }
tail -1 $O/small.log
B="python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
TT2_TR_PERSIST=1 TT2_TP_STAMP=400 TT2_TP_STAMP_FILE=$O/st.bin timeout -k 10 300 $B --train-steps 1 > $O/st.json 2> $O/st.err || { echo "stamp bench failed"; tail -5 $O/st.err; exit 1; }
python scripts/tp_stamps.py $O/st.bin
for m in 1 0; do
  TT2_TR_PERSIST=$m timeout -k 10 300 $B --train-steps 3 > $O/bench_$m.json 2> $O/bench_$m.err || { echo "bench failed $m"; tail -5 $O/bench_$m.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$m.json').read().strip().splitlines()[-1]);t=d['train'];print('persist=$m', t.get('ms_per_step'), t.get('forward_backward_ms'))"
done
timeout -k 10 400 python -u -m pytest tests/test_train.py -x -v -m gpu --timeout 200 --timeout-method thread -k "persistent" -s > $O/persist.log 2>&1 || { echo "persist tests failed"; grep -E "FAILED|Error|frames" $O/persist.log | head -40; tail -30 $O/persist.log; exit 1; }
grep -E "PASSED|frames" $O/persist.log
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/train.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error" $O/train.log | head -20; tail -30 $O/train.log; exit 1; }
tail -2 $O/train.log
TT2_TR_PERSIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2 > $O/prof.json 2> $O/prof.err || { echo "rocprof failed"; tail -5 $O/prof.err; exit 1; }
head -25 $O/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
