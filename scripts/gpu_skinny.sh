# round 3: skinny bf16 GEMM for the training step -- tests, then A/B of the training leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_train.py tests/test_train_options.py -m gpu -q --timeout 200 --timeout-method thread -k "bf16 or full_size or frontend or teacher" > gpurun_out/sk_t.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/sk_t.log
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --no-variants"
TT2_GEMM_SKINNY=0 timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/sk_b0.json 2> gpurun_out/sk_b0.err || exit 1
TT2_GEMM_SKINNY=1 timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/sk_b1.json 2> gpurun_out/sk_b1.err || exit 1
python3 -c "
import json
for f in ('gpurun_out/sk_b0.json','gpurun_out/sk_b1.json'):
    d=json.load(open(f)); t=d['train']; print(f, 'train ms/step', t['ms_per_step'], 'fb', t['forward_backward_ms'], 'decoder', d['value'])
"
