# persistent training forward: stage stamps of step 400 in the configs[4] leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5d
export TMPDIR=/tmp
TT2_TR_PERSIST=1 TT2_TP_STAMP=400 TT2_TP_STAMP_FILE=gpurun_out/r5d/st.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1 > gpurun_out/r5d/b.json 2> gpurun_out/r5d/b.err || { echo "bench failed"; tail -5 gpurun_out/r5d/b.err; exit 1; }
python scripts/tp_stamps.py gpurun_out/r5d/st.bin
