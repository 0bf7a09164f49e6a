# round 4 HEAD verification: full GPU test suite + smoke + default bench + rocprof passes + decoder stage stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_round.sh r04a || exit 1
bash scripts/gpu_r4a.sh
