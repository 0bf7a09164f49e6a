# WaveNet wide generators: parity tests + the wavenet leg of the bench only
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavenet_wide.py tests/test_gpu_wavenet_quantize.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/ww.log 2>&1 || { echo "wide tests failed"; grep -E "FAILED|Error|assert" $O/ww.log | head; tail -20 $O/ww.log; exit 1; }
tail -1 $O/ww.log
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > $O/b.json 2> $O/b.err || { echo "bench failed"; tail -5 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);w=d['wavenet'];print('wn', w['value'], w['us_per_sample']);print({k:(v.get('us_per_sample'), v.get('realtime_factor')) for k,v in w.get('widths',{}).items()})"
