# self-tagged h1/h2/ctx exchange + packed energy puts: persistent / long-horizon / emt parity, then
# decoder A/B (tree vs energy-pack-only vs HEAD) and stage stamps of the tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py tests/test_gpu_emt_attn.py tests/test_gpu_style.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4c/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r4c/tests.log | head -20; tail -30 gpurun_out/r4c/tests.log; exit 1; }
tail -1 gpurun_out/r4c/tests.log
bash scripts/gpu_ab.sh tree variants/lib_pack.so variants/lib_head.so || exit 1
TT2_STAMP_STEP=500 timeout -k 10 150 python bench.py --steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/r4c/st.json 2> gpurun_out/r4c/st.err || { echo "bench failed"; tail -5 gpurun_out/r4c/st.err; exit 1; }
cp gpurun_out/pd_stamps.npy gpurun_out/r4c/pd_stamps.npy
python scripts/stamps.py gpurun_out/r4c/pd_stamps.npy
