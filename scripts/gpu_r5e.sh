# persistent training forward after the asm-load hazard fix: small case, stage stamps of step 400
# at configs[4], A/B of the train leg, then the persistent parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5e
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/dbg_tp_small.py 5 7 3 > gpurun_out/r5e/small.log 2>&1 || { echo "small failed"; tail -5 gpurun_out/r5e/small.log; exit 1; }
tail -1 gpurun_out/r5e/small.log
B="python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
TT2_TR_PERSIST=1 TT2_TP_STAMP=400 TT2_TP_STAMP_FILE=gpurun_out/r5e/st.bin timeout -k 10 300 $B --train-steps 1 > gpurun_out/r5e/st.json 2> gpurun_out/r5e/st.err || { echo "stamp bench failed"; tail -5 gpurun_out/r5e/st.err; exit 1; }
python scripts/tp_stamps.py gpurun_out/r5e/st.bin
for m in 1 0; do
  TT2_TR_PERSIST=$m timeout -k 10 300 $B --train-steps 3 > gpurun_out/r5e/bench_$m.json 2> gpurun_out/r5e/bench_$m.err || { echo "bench failed $m"; tail -5 gpurun_out/r5e/bench_$m.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5e/bench_$m.json').read().strip().splitlines()[-1]);t=d['train'];print('persist=$m', t.get('ms_per_step'), t.get('forward_backward_ms'))"
done
timeout -k 10 400 python -u -m pytest tests/test_train.py -x -v -m gpu --timeout 200 --timeout-method thread -k "persistent" -s > gpurun_out/r5e/persist.log 2>&1 || { echo "persist tests failed"; grep -E "FAILED|Error|frames" gpurun_out/r5e/persist.log | head -40; tail -30 gpurun_out/r5e/persist.log; exit 1; }
grep -E "PASSED|frames" gpurun_out/r5e/persist.log
