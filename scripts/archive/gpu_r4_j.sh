# round 4 j: density-hint first range + chunked hooked passes: tests, forced 1-rank RCCL
# stream with 1 / 4 chunks (+ trace), first-range width variants, 1B / 1e8 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 900 t_j.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grid.py tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_stream.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_forced_dist.py
export LSKNN_DIST_BACKEND=nccl
LSKNN_KNN_CHUNKS=1 run 300 fd_c1.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_KNN_CHUNKS=4 run 300 fd_c4.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_KNN_CHUNKS=8 run 300 fd_c8.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
run 300 fd_c4_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fd3 -o run --output-format csv -- python3 -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
unset LSKNN_DIST_BACKEND
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
run 200 tb_base.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
LSKNN_HIP_LIB=$X/liblsknn_hip_tb8.so run 200 tb_8.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
LSKNN_HIP_LIB=$X/liblsknn_hip_tb12.so run 200 tb_12.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
LSKNN_HIP_LIB=$X/liblsknn_hip_prof.so run 200 cyc3_1e8.log python -u scripts/knn_only.py --points 1e8 --grid 1 --reps 2
run 400 s_1b_j.log python -u bench.py --steps 10 --warmup 3
run 300 s_1e8_j.log python -u bench.py --points 1e8 --steps 20 --warmup 3
