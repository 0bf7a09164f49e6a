# persistent training forward: new tests first, then the training suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train.py -x -v -m gpu --timeout 200 --timeout-method thread -k "persistent" -s > gpurun_out/r5b/persist.log 2>&1 || { echo "persist tests failed"; grep -E "FAILED|Error|error|rel |frames" gpurun_out/r5b/persist.log | head -40; tail -30 gpurun_out/r5b/persist.log; exit 1; }
grep -E "PASSED|frames" gpurun_out/r5b/persist.log
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5b/train.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error" gpurun_out/r5b/train.log | head -20; tail -30 gpurun_out/r5b/train.log; exit 1; }
tail -2 gpurun_out/r5b/train.log
