# train checks (BLAS TN layout, embedding backward) + decoder A/B (tree vs variants/lib_head.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_train_blas.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "persistent" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
bash scripts/gpu_ab.sh tree variants/lib_head.so
