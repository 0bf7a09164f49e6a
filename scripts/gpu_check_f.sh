# (1) pre-session library under poisoned allocations: frontend gradient test; (2) decoder A/B tree vs prefetch variant
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== v0 poison"
TT2_LIB=$GRAFT_REPO_ROOT/variants/lib_v0.so TT2_ALLOC_FILL=255 timeout -k 10 300 python -u -m pytest tests/test_train.py -q -m gpu --timeout 200 --timeout-method thread -k "frontend" > gpurun_out/v0p.log 2>&1
grep -E "passed|failed|^E  .*Assert" gpurun_out/v0p.log | head -3
bash scripts/gpu_ab.sh tree variants/lib_pf.so
