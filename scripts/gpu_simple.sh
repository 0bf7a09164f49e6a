# 'simple' emotion attention in the persistent decoder: emt tests, decoder parity, variants bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_emt_attn.py -x -v -m gpu -k "simple" --timeout 240 --timeout-method thread > $O/sp.log 2>&1 || { echo "simple tests failed"; grep -E "FAILED|Error|assert|Mismatch" $O/sp.log | head -30; tail -30 $O/sp.log; exit 1; }
grep -E "PASSED|FAILED" $O/sp.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_emt_attn.py tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/all.log 2>&1 || { echo "emt/parity tests failed"; tail -30 $O/all.log; exit 1; }
tail -1 $O/all.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train > $O/var.json 2> $O/var.err || { echo "variants bench failed"; tail -5 $O/var.err; exit 1; }
python -c "import json;d=json.loads(open('$O/var.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['us_per_step']);print(json.dumps(d.get('variants'))[:1200])"
