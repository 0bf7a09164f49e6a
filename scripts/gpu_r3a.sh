# round 3: whole -m gpu suite under TT2_REDZONE=1, then one profiled bench with cooperative launches
# (the round-2 exit segfault) with native + Python backtraces on a fatal signal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TT2_REDZONE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/rz3.log 2>&1
echo "redzone suite rc=$?"; tail -3 gpurun_out/rz3.log
export TT2_SEGV_TRACE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seg -o run --output-format csv -- python3 -X faulthandler bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --no-variants > gpurun_out/seg.out 2> gpurun_out/seg.err
echo "prof rc=$?"
tail -5 gpurun_out/seg.out; tail -60 gpurun_out/seg.err
