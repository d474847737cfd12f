# round 4 ab: 10-bit radix passes (3 instead of 4 for 30-bit curve keys) vs 8-bit, tests + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_index_refine.py -k sort"
run 300 ab_t_base.log $T
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort.so run 300 ab_t_wsort.log $T
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort16.so run 300 ab_t_wsort16.log $T
run 200 ab_sb_base.log python -u scripts/sort_bench.py 1e9
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort.so run 200 ab_sb_wsort.log python -u scripts/sort_bench.py 1e9
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort16.so run 200 ab_sb_wsort16.log python -u scripts/sort_bench.py 1e9
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort.so run 300 ab_grid_wsort.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort.so run 420 ab_bench_wsort.log python -u bench.py --gpus 1 --steps 20 --warmup 5
