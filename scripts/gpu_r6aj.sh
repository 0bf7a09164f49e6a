# round 6 (final tree): the whole GPU suite, smoke, the default bench, rocprofv3 kernel stats + PMC passes
# of the decoder / training legs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -40; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-600
bash scripts/gpu_prof.sh r6aj || { echo "prof failed"; exit 1; }

echo done
