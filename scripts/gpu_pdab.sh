# decoder parity tests on the in-tree build, then the decoder A/B (scripts/gpu_ab.sh) against the given libraries
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py tests/test_gpu_emt_attn.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pdab_tests.log 2>&1 || { echo "decoder tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pdab_tests.log | head; tail -30 gpurun_out/pdab_tests.log; exit 1; }
tail -1 gpurun_out/pdab_tests.log
bash scripts/gpu_ab.sh "$@"
