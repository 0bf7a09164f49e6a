# persistent decoder change: parity + long-horizon tests, then A/B decode timing vs variants/dp_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ctxpp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ctxpp_tests.log; exit 1; }
tail -3 gpurun_out/ctxpp_tests.log
bash scripts/gpu_ab.sh tree variants/dp_old.so
