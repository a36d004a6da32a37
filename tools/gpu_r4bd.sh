# r4b then r4d in one call (the pool is short of boxes)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4b.sh || exit 1
bash tools/gpu_r4d.sh || exit 1
