# persistent-decoder change: parity (decoder / emt / long horizon) on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "persistent or parity or longhorizon or emt" > gpurun_out/spill_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/spill_tests.log | head -20; tail -30 gpurun_out/spill_tests.log; exit 1; }
tail -1 gpurun_out/spill_tests.log
