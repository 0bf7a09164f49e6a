# round 6: rocprofv3 kernel trace of the training leg (configs[4]) with the current persistent backward
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2 > $O/prof.json 2> $O/prof.err || { echo "rocprof failed"; tail -5 $O/prof.err; exit 1; }
find $O -name "*.csv" | head
