# round 4 h: where the grid kernel's time goes now — cycle profile (LSK_GRID_PROFILE
# library) and PMC instruction mix of the production kernel, 1e8 uniform, k=100
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
LSKNN_HIP_LIB=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_prof.so run 200 cyc_1e8.log python -u scripts/knn_only.py --points 1e8 --grid 1 --reps 2
run 120 pmc_a.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc_a -o run --output-format csv -- python3 -u scripts/knn_only.py --points 3e7 --grid 1
run 120 pmc_b.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR -d gpurun_out/pmc_b -o run --output-format csv -- python3 -u scripts/knn_only.py --points 3e7 --grid 1
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
for r in 1 2; do
  run 200 ab_base_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
  LSKNN_HIP_LIB=$X/liblsknn_hip_skip1.so run 200 ab_skip1_$r.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
LSKNN_HIP_LIB=$X/liblsknn_hip_skip1.so run 300 ab_skip1_tests.log python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_grid.py
run 600 t_h.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stream.py tests/test_gpu_rccl.py tests/test_forced_dist.py
export LSKNN_DIST_BACKEND=nccl
run 300 fd_1e8_h.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
run 300 fd_1e8_h_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fd2 -o run --output-format csv -- python3 -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
