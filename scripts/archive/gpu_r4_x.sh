# round 4 x: batched histogram shrink A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
LSKNN_HIP_LIB=$X/liblsknn_hip_shrink4.so run 300 x_tests.log python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_grid.py
for r in 1 2; do
  run 200 x_base_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_shrink4.so run 200 x_s4_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
