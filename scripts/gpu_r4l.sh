# decoder A/B: RG1's first recurrent half moved out of the H2 -> query window into the energy
# hand-off's window (rg1: right after the energy puts; rg1b: after the projection h2 partial)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4l
export TMPDIR=/tmp
for L in variants/lib_rg1.so variants/lib_rg1b.so; do
  TT2_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py -x -q -m gpu --timeout 200 --timeout-method thread -k "persistent or longhorizon" > gpurun_out/r4l/t_$(basename $L).log 2>&1 || { echo "tests failed $L"; tail -20 gpurun_out/r4l/t_$(basename $L).log; exit 1; }
  echo "$L $(tail -1 gpurun_out/r4l/t_$(basename $L).log)"
done
bash scripts/gpu_ab.sh tree variants/lib_rg1.so variants/lib_rg1b.so || exit 1
