# training step: parity tests, bench (2 runs), kernel stats (tag = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-t3}
timeout -k 10 400 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_memcheck.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/${TAG}_t.json 2> gpurun_out/${TAG}_t.err || { echo "train bench failed"; tail -5 gpurun_out/${TAG}_t.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_t.json').read().strip().splitlines()[-1]); print('train ms', d['train']['ms_per_step'], d['train']['loss_first'], d['train']['grad_norm'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { echo "prof failed"; tail -5 gpurun_out/${TAG}_prof.err; exit 1; }
head -40 gpurun_out/prof_${TAG}/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-110
