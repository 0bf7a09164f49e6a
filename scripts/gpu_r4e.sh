# prenet hand-off as self-tagged floats (stop bit in bit 1) +/- the L1 context-row loads issued
# before the prenet take (tree: all 8, hov: 4 of 8, pre: none) against the committed r4d build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py -x -q -m gpu --timeout 300 --timeout-method thread -k "persistent or longhorizon or gta or free or stop" > gpurun_out/r4e/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4e/tests.log | head -20; tail -30 gpurun_out/r4e/tests.log; exit 1; }
tail -1 gpurun_out/r4e/tests.log
for L in variants/lib_pre.so variants/lib_hov.so; do
  TT2_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "persistent" > gpurun_out/r4e/t_$(basename $L).log 2>&1 || { echo "tests failed $L"; tail -20 gpurun_out/r4e/t_$(basename $L).log; exit 1; }
  echo "$L $(tail -1 gpurun_out/r4e/t_$(basename $L).log)"
done
bash scripts/gpu_ab.sh tree variants/lib_hov.so variants/lib_pre.so variants/lib_r4d.so || exit 1
TT2_STAMP_STEP=500 timeout -k 10 150 python bench.py --steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/r4e/st.json 2> gpurun_out/r4e/st.err || { echo "bench failed"; tail -5 gpurun_out/r4e/st.err; exit 1; }
cp gpurun_out/pd_stamps.npy gpurun_out/r4e/pd_stamps_tree.npy
python scripts/stamps.py gpurun_out/r4e/pd_stamps_tree.npy
