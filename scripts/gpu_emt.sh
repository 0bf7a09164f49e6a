# Tacotron_emt_attn 'multihead' in the persistent decoder: parity, then the variants bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_emt_attn.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/emt_tests.log 2>&1 || { echo "emt tests failed"; grep -E "PASS|FAIL|Error|assert|Mismatch|max abs" gpurun_out/emt_tests.log | head -40; tail -30 gpurun_out/emt_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/emt_tests.log | cut -c1-120
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k persistent --timeout 150 --timeout-method thread > gpurun_out/emt_par.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/emt_par.log; exit 1; }
tail -1 gpurun_out/emt_par.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train > gpurun_out/emt_b.json 2> gpurun_out/emt_b.err || { echo "bench failed"; tail -5 gpurun_out/emt_b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/emt_b.json').read().strip().splitlines()[-1]); print(d['phases']['decode_us_per_step']); print(json.dumps(d['variants'])[:900])"
