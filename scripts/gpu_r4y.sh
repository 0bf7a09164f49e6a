# energy_bwd2 timing with TT2_TR_VALUES16=0 vs 1 (kernel traces of the training leg only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4y
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2"
for v in 0 1; do
  TT2_TR_VALUES16=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4y/trace$v -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r4y/prof$v.json 2>/dev/null || exit 1
done
echo done
