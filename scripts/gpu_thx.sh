# timing experiment: attention backward staging with / without the tanh-row loads (var/libtt2_x.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for v in base x; do
  L=""
  [ $v = x ] && L="TT2_LIB=$GRAFT_REPO_ROOT/var/libtt2_x.so"
  env $L TT2_ATTQ_STAMP=400 TT2_ATTQ_STAMP_FILE=$O/aq_$v.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-variants --train-steps 2 > $O/aq_$v.json 2> $O/aq_$v.err || { echo "stamp bench failed $v"; tail -5 $O/aq_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/aq_$v.json').read().strip().splitlines()[-1]);t=d['train'];print('$v train', t.get('ms_per_step'))"
  python scripts/attq_stamps.py $O/aq_$v.bin
done
