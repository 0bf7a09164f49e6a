# training-leg check after a train.hip change: GPU training parity tests, then the bench's training leg x2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "train" --timeout 120 --timeout-method thread > gpurun_out/train_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/train_tests.log; exit 1; }
tail -1 gpurun_out/train_tests.log
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --train-steps 3"
for i in 1 2; do
  timeout -k 10 240 python bench.py $ARGS > gpurun_out/tab_$i.json 2> gpurun_out/tab_$i.err || { echo "bench fail"; tail -5 gpurun_out/tab_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/tab_$i.json'));print('run $i', d['value'], d['train']['ms_per_step'], d['train']['loss_last'], d['train']['grad_norm'])"
done
