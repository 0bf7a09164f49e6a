# decoder stage stamps (diagnostic build libtt2_x.so: + store-drain stamp 30) over several launches, per XCD
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2 3; do
  TT2_LIB=$GRAFT_REPO_ROOT/tacotron-2_amd/libtt2_x.so TT2_STAMP_STEP=500 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > $O/stamps$k.json 2> $O/stamps$k.err || { echo "stamp bench failed"; tail -5 $O/stamps$k.err; exit 1; }
  cp gpurun_out/pd_stamps.npy $O/pd_stamps$k.npy && python scripts/stamps.py $O/pd_stamps$k.npy | tail -9
done
