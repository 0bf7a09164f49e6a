# A/B of the wide WaveNet leg of bench.py under each library build given as args (in-tree = "tree")
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > gpurun_out/wab.json 2> gpurun_out/wab.err || { echo "bench failed for $L"; tail -5 gpurun_out/wab.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/wab.json').read().strip().splitlines()[-1]);w=d['wavenet'];print('$L', w['us_per_sample'], {k:v.get('us_per_sample') for k,v in w.get('widths',{}).items()})"
  done
done
