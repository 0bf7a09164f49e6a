# round 6: placement of the persistent forward's off-chain products (TT2_TP_OC A/B) at configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ae
mkdir -p $O
export TMPDIR=/tmp
B="--steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants"
for m in 3; do
  TT2_TP_OC=$m TT2_TP_STAMP=400 TT2_TP_STAMP_FILE=$O/tp400_$m.bin timeout -k 10 300 python -u bench.py $B --train-steps 1 > $O/st$m.json 2> $O/st$m.err || { echo "stamp run failed"; tail -5 $O/st$m.err; exit 1; }
  echo "mode $m"; python scripts/tp_stamps.py $O/tp400_$m.bin
done
for rep in 1 2; do
  for m in 0 1 3; do
    TT2_TP_OC=$m timeout -k 10 300 python -u bench.py $B --train-steps 3 > $O/ab$m.json 2> $O/ab$m.err || { echo "train bench failed"; tail -5 $O/ab$m.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/ab$m.json').read().strip().splitlines()[-1]);t=d['train'];print('oc=$m', t.get('ms_per_step'), t.get('forward_backward_ms'), t.get('grad_norm'))"
  done
done
