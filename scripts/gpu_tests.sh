# GPU parity tests only (tag = $1, optional -k expression = $2)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread $K > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/tests_$TAG.log | head -30; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
