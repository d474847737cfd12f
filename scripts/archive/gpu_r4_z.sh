# round 4 z: collect appends under one exec branch A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
LSKNN_HIP_LIB=$X/liblsknn_hip_flat.so run 300 z_tests.log python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_grid.py
for r in 1 2; do
  run 200 z_base_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_flat.so run 200 z_flat_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
