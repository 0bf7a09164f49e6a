# k_tr_att_bwd_q stage stamps of step 400 (configs[4] train leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
TT2_TR_PERSIST=1 TT2_ATTQ_STAMP=400 TT2_ATTQ_STAMP_FILE=$O/aq.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1 > $O/aq.json 2> $O/aq.err || { echo "bench failed"; tail -5 $O/aq.err; exit 1; }
python scripts/attq_stamps.py $O/aq.bin
