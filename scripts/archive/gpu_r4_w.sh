# round 4 w: band-selection network in the bucket-tree kernel (non-uniform data) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
LSKNN_HIP_LIB=$X/liblsknn_hip_rowsnet.so run 400 w_rowsnet_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "oracle or mixed or heavy or forced or duplicates"
LSK_DISTS=clustered,planar,mixed_scale run 300 w_base.log python -u scripts/dist_robustness.py 20000000 100 16
LSK_DISTS=clustered,planar,mixed_scale LSKNN_HIP_LIB=$X/liblsknn_hip_rowsnet.so run 300 w_rowsnet.log python -u scripts/dist_robustness.py 20000000 100 16
