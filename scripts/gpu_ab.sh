# A/B decoder timing: bench.py decoder leg under each library build given as args (in-tree = "tree")
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed for $L"; tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$L', d['phases']['decode_us_per_step'], d['value'])"
  done
done
