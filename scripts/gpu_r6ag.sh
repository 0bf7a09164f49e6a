# round 6: kernel trace of the training step with the direct refnet conv2d backward
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2 > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -5 $O/prof.err; exit 1; }
python scripts/train_step_kernels.py $O/prof/run_kernel_trace.csv 30
python - <<'PY'
import csv
rows = sorted(csv.DictReader(open('gpurun_out/r6ag/prof/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
adam = [i for i, r in enumerate(rows) if 'k_tr_adam' in r['Kernel_Name']]
for r in rows[adam[-2] + 1: adam[-1] + 1]:
    if 'conv2d' in r['Kernel_Name']:
        print("%8.1f us %s grid %s" % ((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, r['Kernel_Name'].split('(')[0][-28:], r['Grid_Size_X']))
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train.py -k "refnet_conv_backward or frontend" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 3"
for rep in 1 2; do
  for d in 0 1; do :
    TT2_FE_CONV_DIRECT=$d timeout -k 10 300 python -u bench.py $B > $O/ab.json 2> $O/ab.err || { echo "train bench failed"; tail -5 $O/ab.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);t=d['train'];print('direct=$d', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'))"
  done
done
