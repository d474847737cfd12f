#!/bin/bash
# Cycle profile of the grid kernel (LSK_GRID_PROFILE build "prof"): hist / collect
# evaluations per query and the share of wave time per phase, 1e7 and 1e8 uniform, k = 100.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r6_prof.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_prof.so python scripts/knn_ab.py --points 1e7 1e8 --k 100 --reps 2 || exit $?
cat gpurun_out/r6_prof.log
