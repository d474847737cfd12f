# grandchild culling by the union of the wave's 4 row regions (rowcull = LSK_GRID_ROWCULL=1)
# vs the wave box (base): grid tests, k-NN pass at 1e8, then the 1B bench on rowcull
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in rowcull base; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 300 rc_tests_$v.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_grid.py
  grep -q " passed" gpurun_out/rc_tests_$v.log && ! grep -q "failed" gpurun_out/rc_tests_$v.log || exit 1
  LSKNN_HIP_LIB=$L run 300 rc_knn_$v.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
LSKNN_HIP_LIB=$X/liblsknn_hip_rowcull.so run 500 rc_bench_1b.log python -u bench.py --gpus 1 --steps 20 --warmup 5
