# round 6 first call: the status-word test + persistent training tests, then the configs[4] loss
# trajectory diagnostic
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_train.py \
  -k "failed_persistent or persistent_forward or full_size" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -8 $O/tests.log
timeout -k 10 900 python -u scripts/diag_train_loss.py --steps 6 > $O/diag_loss.jsonl 2> $O/diag.err || { echo "diag failed"; tail -20 $O/diag.err; exit 1; }
cat $O/diag_loss.jsonl
