# round-4 full cycle: GPU tests, smoke, default bench, rocprof kernel trace + PMC passes (decoder +
# training), a kernel trace WITH the WaveNet legs (k_generate_pipe / k_generate_wide), stage stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r04b}
bash scripts/gpu_round.sh $TAG || exit 1
mkdir -p gpurun_out/wn_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/wn_$TAG/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-train --no-e2e --no-griffin-lim --no-variants > gpurun_out/wn_$TAG/bench.json 2> gpurun_out/wn_$TAG/bench.err || { echo "wavenet trace failed"; tail -5 gpurun_out/wn_$TAG/bench.err; exit 1; }
echo "wavenet trace ok"
TT2_STAMP_STEP=500 timeout -k 10 150 python bench.py --steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/st_$TAG.json 2> gpurun_out/st_$TAG.err || { echo "stamps failed"; exit 1; }
cp gpurun_out/pd_stamps.npy gpurun_out/pd_stamps_$TAG.npy
python scripts/stamps.py gpurun_out/pd_stamps_$TAG.npy
