# round 6: persistent backward with the next step's HBM operands prefetched in the off-chain window: the training test
# files, stamps, A/B against the per-step launches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp
TT2_TB_STAMP=400 TT2_TB_STAMP_FILE=$O/tb400.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1 > $O/st.json 2> $O/st.err || { echo "stamp run failed"; tail -5 $O/st.err; exit 1; }
python scripts/tb_stamps.py $O/tb400.bin
