#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in b48t8 b48t12 b40t8 b44t10; do
LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so LSK_ROWS_RCAP=32 run 300 knn_${v}.log python scripts/knn_only.py --points 1e8 --reps 2 --impl rows
done
