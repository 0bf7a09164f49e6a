# attention backward changes: training suites, train leg, attq stage stamps; emt DPP changes: emt tests + variants
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_train_options.py tests/test_gpu_train_api.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/train.log 2>&1 || { echo "train tests failed"; grep -E "FAILED|Error|assert" $O/train.log | head -20; tail -30 $O/train.log; exit 1; }
tail -1 $O/train.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);t=d['train'];print('train', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'))"
TT2_ATTQ_STAMP=400 TT2_ATTQ_STAMP_FILE=$O/aq.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 1 > $O/aq.json 2> $O/aq.err || { echo "stamp bench failed"; tail -5 $O/aq.err; exit 1; }
python scripts/attq_stamps.py $O/aq.bin
timeout -k 10 500 python -u -m pytest tests/test_gpu_emt_attn.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/emt.log 2>&1 || { echo "emt tests failed"; grep -E "FAILED|Error|assert" $O/emt.log | head; tail -20 $O/emt.log; exit 1; }
tail -1 $O/emt.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train > $O/var.json 2> $O/var.err || { echo "variants bench failed"; tail -5 $O/var.err; exit 1; }
python -c "import json;d=json.loads(open('$O/var.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['us_per_step']);v=d['variants'];print({k:v[k].get('decode_us_per_step') for k in v})"
