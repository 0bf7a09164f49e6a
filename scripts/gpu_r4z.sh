# R = 256 one-hop WaveNet generator: wide parity tests, widths A/B (TT2_WW_ONEHOP=1 vs 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4z
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_wavenet_wide.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4z/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error|^E " gpurun_out/r4z/tests.log | head -20; tail -30 gpurun_out/r4z/tests.log; exit 1; }
tail -1 gpurun_out/r4z/tests.log
ARGS="--steps 1 --warmup 1 --no-train --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
for v in 1 0; do
  TT2_WW_ONEHOP=$v timeout -k 10 400 python bench.py $ARGS > gpurun_out/r4z/b$v.json 2> gpurun_out/r4z/b$v.err || { echo "bench failed"; tail -5 gpurun_out/r4z/b$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4z/b$v.json').read().strip().splitlines()[-1]); w=d['wavenet']['widths']; print('onehop=$v', w['paper_r256']['us_per_sample'], w['paper_r256']['realtime_factor'], w['fork_r128']['us_per_sample'])"
done
