# round 3: wide WaveNet (R=128 / R=256 two-hop) parity + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wavenet_wide.py tests/test_gpu_wavenet_variants.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/wide_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/wide_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-griffin-lim --no-variants --no-train > gpurun_out/wide_b.json 2> gpurun_out/wide_b.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/wide_b.json'))['wavenet']
print('R64', d['value'], d['us_per_sample'], 'batch', d.get('batch'))
for k,v in d['widths'].items(): print(k, v['value'], v['us_per_sample'], v['realtime_factor'])
"
