# front-end conv backward kernels: training suites, train leg, kernel trace of the train leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/train.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error|assert" $O/train.log | head -20; tail -30 $O/train.log; exit 1; }
tail -2 $O/train.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);t=d['train'];print('train', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'))"
bash scripts/gpu_prof_train.sh $1 | head -30
TT2_STAMP_STEP=500 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --no-train > $O/stamps.json 2> $O/stamps.err || { echo "stamp bench failed"; tail -5 $O/stamps.err; exit 1; }
cp gpurun_out/pd_stamps.npy $O/pd_stamps.npy && python scripts/stamps.py $O/pd_stamps.npy
