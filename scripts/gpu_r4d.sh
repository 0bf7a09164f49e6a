# tagged h2 / ctx hand-offs with the h1 protocol as an A/B switch (tree: drained flag; h1t1: tags +
# flag hint; h1t2: tags + data polling) against the energy-pack-only build; parity of the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py tests/test_gpu_emt_attn.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4d/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4d/tests.log | head -20; tail -30 gpurun_out/r4d/tests.log; exit 1; }
tail -1 gpurun_out/r4d/tests.log
bash scripts/gpu_ab.sh tree variants/lib_h1t1.so variants/lib_h1t2.so variants/lib_pack.so || exit 1
for L in tree variants/lib_h1t2.so; do
  if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
  TT2_STAMP_STEP=500 timeout -k 10 150 python bench.py --steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/r4d/st.json 2> gpurun_out/r4d/st.err || { echo "bench failed"; tail -5 gpurun_out/r4d/st.err; exit 1; }
  echo "== stamps $L"; python scripts/stamps.py gpurun_out/pd_stamps.npy
done
