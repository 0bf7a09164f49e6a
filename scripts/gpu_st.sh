# style_tokens in the persistent decoder + front-end conv kernels + decoder XCD stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_emt_attn.py -x -v -m gpu -k "style_tokens" --timeout 240 --timeout-method thread > $O/st.log 2>&1 || { echo "style_tokens tests failed"; grep -E "FAILED|Error|assert|Mismatch" $O/st.log | head -30; tail -30 $O/st.log; exit 1; }
grep -E "PASSED|FAILED" $O/st.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_emt_attn.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/emt.log 2>&1 || { echo "emt tests failed"; tail -30 $O/emt.log; exit 1; }
tail -2 $O/emt.log
bash scripts/gpu_fe.sh $1
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train > $O/var.json 2> $O/var.err || { echo "variants bench failed"; tail -5 $O/var.err; exit 1; }
python -c "import json;d=json.loads(open('$O/var.json').read().strip().splitlines()[-1]);print(json.dumps(d.get('variants'))[:900])"
