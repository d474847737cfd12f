set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
LSKNN_KNN_CHUNKS=1 LSKNN_DIST_BACKEND=nccl run 300 dbg_hook2.log python -u scripts/debug_hook.py 1e8
