# round 4 u: band selection by a sorting network (16 / 32 values) vs the LDS heap
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
LSKNN_HIP_LIB=$X/liblsknn_hip_net32.so run 300 u_net32_tests.log python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_grid.py
for r in 1 2; do
  run 200 u_base_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_net32.so run 200 u_net32_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_net16.so run 200 u_net16_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
