# emt persistent: parity subset, stage stamps, variants bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_emt_attn.py -x -q -m gpu -k "persistent" --timeout 200 --timeout-method thread > gpurun_out/emt2_tests.log 2>&1 || { echo "emt tests failed"; tail -30 gpurun_out/emt2_tests.log; exit 1; }
tail -1 gpurun_out/emt2_tests.log
timeout -k 10 200 python scripts/emt_stamps.py > gpurun_out/emt_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/emt_stamps.txt; exit 1; }
cat gpurun_out/emt_stamps.txt
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train > gpurun_out/emt_b.json 2> gpurun_out/emt_b.err || { echo "bench failed"; tail -5 gpurun_out/emt_b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/emt_b.json').read().strip().splitlines()[-1]); print(d['phases']['decode_us_per_step']); v=d['variants']; print({k: v[k].get('decode_us_per_step') for k in v})"
