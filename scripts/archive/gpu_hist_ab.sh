# branch-free paired-lane histogram (default now) vs the exec-masked one (oldhist) and a
# 6-waves/SIMD register budget (minw6): grid tests, k-NN pass at 1e8, then the 1B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
run 300 hist_gridtests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_grid.py tests/test_gpu_kernels.py
grep -q " passed" gpurun_out/hist_gridtests.log && ! grep -q "failed" gpurun_out/hist_gridtests.log || exit 1
for v in base oldhist minw6; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 300 hist_knn_$v.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
run 500 hist_bench.log python -u bench.py --gpus 1 --steps 20 --warmup 5
