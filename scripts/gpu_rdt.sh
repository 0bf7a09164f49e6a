# A/B of the register-direct GEMM's work-group target (TT2_RD_TARGET) on the training step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in 256 160 200 256 128; do
  TT2_RD_TARGET=$cfg timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/rdt.json 2> gpurun_out/rdt.err || { echo "bench failed"; tail -5 gpurun_out/rdt.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/rdt.json').read().strip().splitlines()[-1]); print('target $cfg', d['train']['ms_per_step'])"
done
