# persistent training forward: parity tests, then the configs[4] leg A/B (TT2_TR_PERSIST=1/0) and a
# kernel trace of the persistent step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5c
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train.py -x -v -m gpu --timeout 200 --timeout-method thread -k "persistent" -s > gpurun_out/r5c/persist.log 2>&1 || { echo "persist tests failed"; grep -E "FAILED|Error|frames" gpurun_out/r5c/persist.log | head -40; tail -30 gpurun_out/r5c/persist.log; exit 1; }
grep -E "PASSED|frames" gpurun_out/r5c/persist.log
B="python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for m in 1 0 1; do
  TT2_TR_PERSIST=$m timeout -k 10 300 $B > gpurun_out/r5c/bench_$m.json 2> gpurun_out/r5c/bench_$m.err || { echo "bench failed $m"; tail -5 gpurun_out/r5c/bench_$m.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5c/bench_$m.json').read().strip().splitlines()[-1]);t=d['train'];print('persist=$m', t.get('ms_per_step'), t.get('value'))"
done
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5c/train.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error" gpurun_out/r5c/train.log | head -20; tail -30 gpurun_out/r5c/train.log; exit 1; }
tail -2 gpurun_out/r5c/train.log
