# round 4 q: batch-level skip in the histogram / collect passes (A/B, k-NN alone at 1e8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
for r in 1 2; do
  run 200 q_base_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_noskip4.so run 200 q_ns4_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_noskip4c.so run 200 q_ns4c_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
