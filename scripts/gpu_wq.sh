# mulaw-quantize / unconditional WaveNet tests, then the existing WaveNet parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_wavenet_quantize.py -x -v -m gpu --timeout 240 --timeout-method thread > $O/wq.log 2>&1 || { echo "wq tests failed"; grep -E "FAILED|Error|assert|Mismatch" $O/wq.log | head -30; tail -40 $O/wq.log; exit 1; }
grep -E "PASSED|FAILED" $O/wq.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wavenet_wide.py -x -q -m gpu -k "wavenet or wide" --timeout 240 --timeout-method thread > $O/wn.log 2>&1 || { echo "wn tests failed"; tail -30 $O/wn.log; exit 1; }
tail -2 $O/wn.log
