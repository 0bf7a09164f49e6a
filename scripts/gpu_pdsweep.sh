# persistent decoder: poll back-off sweep (bench only, decoder only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sw}
for S in ${SWEEP:-0 1 2 4 8}; do
  env ${SWVAR:-TT2_PD_SLEEP}=$S timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-wavenet > gpurun_out/sw_${TAG}_$S.json 2> gpurun_out/sw_${TAG}_$S.err || { echo "bench failed $S"; tail -5 gpurun_out/sw_${TAG}_$S.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sw_${TAG}_$S.json')); print($S, d['roofline']['us_per_step'])"
done
