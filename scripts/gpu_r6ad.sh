# round 6: persistent training forward stage stamps (step 400 and 10) at configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ad
mkdir -p $O
export TMPDIR=/tmp
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1"
TT2_TP_STAMP=400 TT2_TP_STAMP_FILE=$O/tp400.bin timeout -k 10 300 python -u bench.py $B > $O/st.json 2> $O/st.err || { echo "stamp run failed"; tail -5 $O/st.err; exit 1; }
python scripts/tp_stamps.py $O/tp400.bin
TT2_TP_STAMP=10 TT2_TP_STAMP_FILE=$O/tp10.bin timeout -k 10 300 python -u bench.py $B > $O/st2.json 2> $O/st2.err || { echo "stamp run failed"; tail -5 $O/st2.err; exit 1; }
python scripts/tp_stamps.py $O/tp10.bin
