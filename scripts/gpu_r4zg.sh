# redzone pass over the round-4 kernels: planes convs (inference + training), gemm_bf16_kc, the
# one-hop WaveNet -- every DevBuf gets a guard band checked after each ABI call (TT2_REDZONE=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4zg
export TMPDIR=/tmp
export TT2_REDZONE=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wavenet_wide.py tests/test_train.py -x -q -m gpu -k "postnet or encoder or full_dims or paper or fork or planes or gathered or library or fused" --timeout 600 --timeout-method thread > gpurun_out/r4zg/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r4zg/tests.log | head; tail -20 gpurun_out/r4zg/tests.log; exit 1; }
tail -1 gpurun_out/r4zg/tests.log
