# round 4 baseline: stage stamps of k_decode_persist at step 500 (3 reps), then a PMC-free kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
for rep in 1 2 3; do
  TT2_STAMP_STEP=500 timeout -k 10 150 python bench.py --steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/r4a/st$rep.json 2> gpurun_out/r4a/st$rep.err || { echo "bench failed"; tail -5 gpurun_out/r4a/st$rep.err; exit 1; }
  cp gpurun_out/pd_stamps.npy gpurun_out/r4a/pd_stamps$rep.npy
  python -c "import json; d=json.loads(open('gpurun_out/r4a/st$rep.json').read().strip().splitlines()[-1]); print(d['phases']['decode_us_per_step'])"
  python scripts/stamps.py gpurun_out/r4a/pd_stamps$rep.npy
done
