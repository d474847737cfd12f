# round 4 aa: 6 waves/SIMD register budget (no spills) vs 7 (spills) for the final kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
for r in 1 2; do
  run 200 aa_base_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_minw6.so run 200 aa_minw6_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
