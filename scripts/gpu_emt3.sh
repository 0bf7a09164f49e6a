# emt persistent stage stamps only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/emt_stamps.py > gpurun_out/emt_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/emt_stamps.txt; exit 1; }
cat gpurun_out/emt_stamps.txt
