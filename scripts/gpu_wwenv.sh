# wide WaveNet parity tests, then the wavenet bench leg under each "VAR=value" env setting given as args ("-" = none)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavenet_wide.py tests/test_gpu_wavenet_quantize.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/wwenv_tests.log 2>&1 || { echo "wide tests failed"; grep -E "FAILED|Error|assert" gpurun_out/wwenv_tests.log | head; tail -30 gpurun_out/wwenv_tests.log; exit 1; }
tail -1 gpurun_out/wwenv_tests.log
for rep in 1 2; do
  for E in "$@"; do
    timeout -k 10 300 env $([ "$E" = "-" ] || echo "$E") python -u bench.py --steps 1 --warmup 1 --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > gpurun_out/wenv.json 2> gpurun_out/wenv.err || { echo "bench failed for $E"; tail -5 gpurun_out/wenv.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/wenv.json').read().strip().splitlines()[-1]);w=d['wavenet'];print('$E', w['us_per_sample'], {k:v.get('us_per_sample') for k,v in w.get('widths',{}).items()})"
  done
done
