# rocprofv3: kernel-trace stats + separate PMC passes (never combined with trace domains)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
# cooperative launches as in the product; bench.py installs tt2_exit_guard under rocprofv3 (the HIP
# runtime's exit-time teardown of the cooperative queue faults after the profiler finalised)
TAG=${1:-p}
ARGS="${PROF_ARGS:---steps 1 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --no-variants}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.bench.json 2>/dev/null && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$TAG/fetch -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$TAG/write -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof_$TAG/tcc -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/prof_$TAG/sq -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2>&1
echo rc=$?
find gpurun_out/prof_$TAG -name "*.csv" | head -20
