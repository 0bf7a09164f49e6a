# decoder micro-change: parity (persistent tests) + production / floor step times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "persistent or full_dims or long" --timeout 240 --timeout-method thread > $O/par.log 2>&1 || { echo "parity failed"; grep -E "FAILED|Error|assert|Mismatch" $O/par.log | head; tail -20 $O/par.log; exit 1; }
tail -1 $O/par.log
timeout -k 10 300 python -u scripts/pd_floor.py > $O/prod.log 2>&1 || { echo "prod failed"; tail -5 $O/prod.log; exit 1; }
tail -1 $O/prod.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > $O/b.json 2> $O/b.err || { echo "bench failed"; tail -5 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['roofline']['us_per_step'])"
timeout -k 10 500 python -u -m pytest tests/test_gpu_emt_attn.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/emt.log 2>&1 || { echo "emt failed"; grep -E "FAILED|Error|assert" $O/emt.log | head; tail -20 $O/emt.log; exit 1; }
tail -1 $O/emt.log
