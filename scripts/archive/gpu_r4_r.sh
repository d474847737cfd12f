# round 4 r: key census occupancy; 1B kernel trace (build time per set)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 300 t_r.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grid.py tests/test_gpu_kernels.py -k "census or level or grid"
run 500 s1b_r_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1b_r -o run --output-format csv -- python3 -u bench.py --steps 4 --warmup 2
run 200 sortb_base.log python -u scripts/sort_bench.py 1e9
LSKNN_HIP_LIB=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_rows8.so run 200 sortb_rows8.log python -u scripts/sort_bench.py 1e9
