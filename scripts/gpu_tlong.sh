# persistent decoder at T_in > 256: new long-input tests, then every persistent/decoder parity test, then a quick bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "long_inputs" --timeout 240 --timeout-method thread > $O/tl.log 2>&1 || { echo "long-input tests failed"; grep -E "FAILED|Error|assert|Mismatch|timed out" $O/tl.log | head -30; tail -40 $O/tl.log; exit 1; }
grep -E "PASSED|FAILED" $O/tl.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/par.log 2>&1 || { echo "parity tests failed"; tail -30 $O/par.log; exit 1; }
tail -2 $O/par.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['us_per_step'])"
