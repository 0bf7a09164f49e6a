# fp32-output 256 x 256 kernel for the BiLSTM input projection: A/B against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4zf
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train"
for rep in 1 2 3; do
  for L in tree variants/lib_prev.so; do
    if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4zf/b.json 2> gpurun_out/r4zf/b.err || { echo "bench failed"; tail -5 gpurun_out/r4zf/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4zf/b.json').read().strip().splitlines()[-1]); print('$L', d['value'], d['phases'])"
  done
done
