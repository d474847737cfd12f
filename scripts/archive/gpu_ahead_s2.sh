# next set's build beside the current k-NN (LSKNN_BUILD_AHEAD=1) with the branch-free grid
# kernel, against the default (build between the k-NN kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
for c in 1 0; do
  LSKNN_BUILD_AHEAD=$c run 400 ahead2_1b_$c.log python -u bench.py --steps 8 --warmup 2 --verify 64
done
