# training: library-GEMM path tests + bench train leg with TT2_TRAIN_BLAS=1 (default) vs 0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train.py -x -q -m gpu --timeout 300 --timeout-method thread -k "bf16 or full_size or frontend" > gpurun_out/tb.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tb.log; exit 1; }
tail -2 gpurun_out/tb.log
for f in 1 0; do
  TT2_TRAIN_BLAS=$f timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants > gpurun_out/tbb_$f.json 2> gpurun_out/tbb_$f.err || { echo "bench failed"; tail -20 gpurun_out/tbb_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/tbb_$f.json').read().strip().splitlines()[-1]); t=d['train']; print('BLAS=$f', t['ms_per_step'], t['loss_first'], t['loss_last'], t['grad_norm'])"
done
