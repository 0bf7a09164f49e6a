# round-3 batch: decoder CTX granules, row attention kernels (training), register-direct GEMM (opt-in)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py tests/test_train.py tests/test_train_options.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
TT2_GEMM_SKINNY=2 timeout -k 10 300 python -u -m pytest tests/test_train.py -x -q -m gpu -k "bf16 or full_size" --timeout 150 --timeout-method thread > gpurun_out/r3b_rd.log 2>&1 || { echo "rd tests failed"; tail -30 gpurun_out/r3b_rd.log; exit 1; }
tail -2 gpurun_out/r3b_rd.log
D="python bench.py --steps 3 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants"
for L in tree variants/dp_old.so tree variants/dp_old.so; do
  if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
  timeout -k 10 120 $D > gpurun_out/r3b_d.json 2> gpurun_out/r3b_d.err || { echo "dec bench failed $L"; tail -5 gpurun_out/r3b_d.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r3b_d.json').read().strip().splitlines()[-1]); print('$L', d['phases']['decode_us_per_step'])"
done
unset TT2_LIB

for cfg in "TT2_TR_ATT_ROW=0" "TT2_TR_ATT_ROW=1" "TT2_GEMM_SKINNY=2"; do
  env $cfg timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/r3b_t.json 2> gpurun_out/r3b_t.err || { echo "train bench failed $cfg"; tail -5 gpurun_out/r3b_t.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r3b_t.json').read().strip().splitlines()[-1]); print('$cfg', d['train']['ms_per_step'])"
done
TT2_GEMM_SKINNY=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/r3b_prof.json 2> gpurun_out/r3b_prof.err || { echo "prof failed"; tail -5 gpurun_out/r3b_prof.err; exit 1; }
head -24 gpurun_out/prof_r3b/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-110
