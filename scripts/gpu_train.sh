# training leg: bench (configs[4]) + rocprof kernel stats (tag = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
ARGS="--no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --steps 1 --warmup 1 ${TRAIN_ARGS}"
timeout -k 10 600 python bench.py $ARGS > gpurun_out/train_$TAG.json 2> gpurun_out/train_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/train_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/train_$TAG.json')); print(json.dumps(d['train']))"
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_$TAG -o run --output-format csv -- python bench.py $ARGS --train-steps 1 > gpurun_out/train_prof_$TAG.json 2> gpurun_out/train_prof_$TAG.err || { echo "prof failed"; tail -20 gpurun_out/train_prof_$TAG.err; exit 1; }
fi
echo done
