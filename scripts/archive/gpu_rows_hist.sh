# branch-free paired-lane histogram in the bucket-tree kernel (knn_rows, default now) vs the
# exec-masked one (rowsold): GPU tests on the default, tree k-NN pass at 1e8, non-uniform
# robustness at 2e7 (those sets take the tree kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
run 600 rh_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_grid.py tests/test_gpu_distributed.py tests/test_index_refine.py -m gpu
grep -q " passed" gpurun_out/rh_tests.log && ! grep -q "failed" gpurun_out/rh_tests.log || exit 1
for v in base rowsold; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 300 rh_knn_$v.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 0
  LSKNN_HIP_LIB=$L run 400 rh_robust_$v.log python -u scripts/dist_robustness.py 20000000 100 16
done
