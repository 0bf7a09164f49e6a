# (1) decoder A/B tree vs prefetch variant (+ its persistent parity tests); (2) pre-session library
# under poisoned allocations: front-end gradient test
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TT2_LIB=$GRAFT_REPO_ROOT/variants/lib_pf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "persistent" > gpurun_out/pf.log 2>&1; tail -1 gpurun_out/pf.log
bash scripts/gpu_ab.sh tree variants/lib_pf.so || exit 1
echo "== v0 poison"
TT2_LIB=$GRAFT_REPO_ROOT/variants/lib_v0.so TT2_ALLOC_FILL=255 timeout -k 10 300 python -u -m pytest tests/test_train.py -q -m gpu --timeout 200 --timeout-method thread -k "frontend" > gpurun_out/v0p.log 2>&1
grep -E "passed|failed|^E  .*Assert" gpurun_out/v0p.log | head -3
