# round 6: the new training tests (configs[4] fp32/bf16 + oracle trajectory, smoothing, status word)
# and the WaveNet Synthesizer's unconditional / debug paths
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_train_options.py tests/test_gpu_wavenet_quantize.py tests/test_train.py \
  -k "smoothing or synthesizer or configs4 or failed_persistent" > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|^1 |^2 |^3 |fp32|bf16" $O/tests.log | tail -30
