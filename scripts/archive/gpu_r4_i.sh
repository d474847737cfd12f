# round 4 i: host timeline of the forced 1-rank stream; cycle profile with the finer
# markers; first-range-from-hint variant A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
LSKNN_DIST_BACKEND=nccl run 300 dbg_hook.log python -u scripts/debug_hook.py 1e8
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
LSKNN_HIP_LIB=$X/liblsknn_hip_prof.so run 200 cyc2_1e8.log python -u scripts/knn_only.py --points 1e8 --grid 1 --reps 2
for r in 1 2; do
  run 200 ab2_base_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_esthint.so run 200 ab2_esthint_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
LSKNN_HIP_LIB=$X/liblsknn_hip_esthint.so run 300 ab2_esthint_tests.log python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_grid.py
