# persistent-decoder poll back-off sweep (TT2_PD_SLEEP = s_sleep(1) repeats between polls)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in "$@"; do
  TT2_PD_SLEEP=$s timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo "bench failed for $s"; tail -5 gpurun_out/sw.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('sleep $s', d['phases']['decode_us_per_step'])"
done
