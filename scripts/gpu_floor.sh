# decoder: production vs arithmetic-free floor instance, plus the floor's stage stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/pd_floor.py > $O/prod.log 2>&1 || { echo "prod failed"; tail -5 $O/prod.log; exit 1; }
tail -1 $O/prod.log
TT2_PD_FLOOR=1 timeout -k 10 300 python -u scripts/pd_floor.py > $O/floor.log 2>&1 || { echo "floor failed"; tail -5 $O/floor.log; exit 1; }
tail -1 $O/floor.log
TT2_PD_FLOOR=1 TT2_STAMP_STEP=500 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > $O/fst.json 2> $O/fst.err || { echo "floor stamps failed"; tail -5 $O/fst.err; exit 1; }
cp gpurun_out/pd_stamps.npy $O/pd_stamps_floor.npy && python scripts/stamps.py $O/pd_stamps_floor.npy | head -23
