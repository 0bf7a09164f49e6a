# WaveNet parity tests (every WaveNet GPU test file) on the in-tree build, then the wavenet bench leg under each library (in-tree = "tree"), 3 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_wavenet_wide.py tests/test_gpu_wavenet_quantize.py tests/test_gpu_wavenet_variants.py tests/test_gpu_parity.py tests/test_gpu_e2e.py tests/test_gpu_longhorizon.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/wwlib_tests.log 2>&1 || { echo "wavenet tests failed"; grep -E "FAILED|Error|assert" gpurun_out/wwlib_tests.log | head; tail -30 gpurun_out/wwlib_tests.log; exit 1; }
tail -1 gpurun_out/wwlib_tests.log
for rep in 1 2 3; do
  for L in "$@"; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > gpurun_out/wlib.json 2> gpurun_out/wlib.err || { echo "bench failed for $L"; tail -5 gpurun_out/wlib.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/wlib.json').read().strip().splitlines()[-1]);w=d['wavenet'];print('$L', w['us_per_sample'], w['batch']['us_per_sample'], {k:v.get('us_per_sample') for k,v in w.get('widths',{}).items()})"
  done
done
