# measurement plumbing: the HBM copy test, then one default bench line (decoder + WaveNet rooflines)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_measure.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/meas_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/meas_tests.log; exit 1; }
tail -1 gpurun_out/meas_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-train --no-variants --no-e2e --no-griffin-lim > gpurun_out/meas_b.json 2> gpurun_out/meas_b.err || { echo "bench failed"; tail -5 gpurun_out/meas_b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/meas_b.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['frac'], r['peak_measured'], r['frac_of_measured']); print(d['wavenet']['roofline'])"
