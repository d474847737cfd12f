#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
run 600 tk.log python -m pytest tests/test_gpu_kernels.py -q -m gpu -x
run 300 knn_rows.log python scripts/knn_only.py --points 1e8 --reps 2 --impl rows
LSKNN_HIP_LIB=$L/liblsknn_hip_prof.so run 300 prof.log python scripts/knn_only.py --points 1e8 --reps 1 --impl rows
