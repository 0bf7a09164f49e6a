# stage stamps of k_decode_persist (step 500) for the in-tree build and each variant library given
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in tree "$@"; do
  if [ "$L" = "tree" ]; then unset TT2_LIB; else export TT2_LIB=$GRAFT_REPO_ROOT/$L; fi
  TT2_STAMP_STEP=500 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-wavenet --no-e2e --no-griffin-lim --no-cpu-baseline --no-train --no-variants > gpurun_out/st.json 2> gpurun_out/st.err || { echo "bench failed for $L"; tail -5 gpurun_out/st.err; exit 1; }
  echo "== $L"; python -c "import json; d=json.loads(open('gpurun_out/st.json').read().strip().splitlines()[-1]); print(d['phases']['decode_us_per_step'])"
  python scripts/stamps.py gpurun_out/pd_stamps.npy
done
