# AdaIN / pretrained_emb_disc_all training + AdaIN inference (separate emotion conv weights) + long-input timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_train.py tests/test_gpu_train_api.py -x -v -m gpu -k "adain or pretrained" --timeout 240 --timeout-method thread > $O/ad.log 2>&1 || { echo "adain tests failed"; grep -E "FAILED|Error|assert|rel" $O/ad.log | head -30; tail -30 $O/ad.log; exit 1; }
grep -E "PASSED|FAILED" $O/ad.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_style.py tests/test_gpu_train_api.py tests/test_train.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/st.log 2>&1 || { echo "style/train tests failed"; tail -30 $O/st.log; exit 1; }
tail -2 $O/st.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s -m gpu -k "long_inputs_match_launch" --timeout 240 --timeout-method thread > $O/tl.log 2>&1 || { echo "long test failed"; tail -20 $O/tl.log; exit 1; }
grep -E "us/step|PASSED" $O/tl.log
