# round 6: persistent backward stage stamps (step 400 of the configs[4] step) + rocprof kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp
TT2_TR_PERSIST_BWD=1 TT2_TB_STAMP=400 TT2_TB_STAMP_FILE=$O/tb400.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1 > $O/st.json 2> $O/st.err || { echo "stamp run failed"; tail -5 $O/st.err; exit 1; }
python scripts/tb_stamps.py $O/tb400.bin
TT2_TR_PERSIST_BWD=1 TT2_TB_STAMP=10 TT2_TB_STAMP_FILE=$O/tb10.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1 > $O/st2.json 2> $O/st2.err || { echo "stamp run failed"; tail -5 $O/st2.err; exit 1; }
python scripts/tb_stamps.py $O/tb10.bin
TT2_TR_PERSIST_BWD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -25 "$f"
