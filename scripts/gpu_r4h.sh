# decoder A/B: the projection blocks' RG2 first-half tail moved after their prenet hand-off (rg2p) or
# every work-group's (rg2a), against the tree; persistent parity of both variants first
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4h
export TMPDIR=/tmp
for L in variants/lib_rg2p.so variants/lib_rg2a.so; do
  TT2_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py -x -q -m gpu --timeout 200 --timeout-method thread -k "persistent or longhorizon" > gpurun_out/r4h/t_$(basename $L).log 2>&1 || { echo "tests failed $L"; tail -20 gpurun_out/r4h/t_$(basename $L).log; exit 1; }
  echo "$L $(tail -1 gpurun_out/r4h/t_$(basename $L).log)"
done
bash scripts/gpu_ab.sh tree variants/lib_rg2p.so variants/lib_rg2a.so || exit 1
