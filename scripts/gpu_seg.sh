# round 3: the rocprofv3 exit segfault with cooperative launches -- exit guard, then a PMC pass
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seg -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --no-variants > gpurun_out/seg.out 2> gpurun_out/seg.err
echo "prof coop+guard rc=$?"
tail -2 gpurun_out/seg.err; ls -la gpurun_out/prof_seg
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_seg_w -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --no-variants --no-train > gpurun_out/segw.out 2> gpurun_out/segw.err
echo "pmc coop+guard rc=$?"
ls -la gpurun_out/prof_seg_w
