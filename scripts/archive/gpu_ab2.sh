#!/bin/bash
# A/B of kernel library variants (lib/exp/liblsknn_hip_<v>.so): k-NN kernel alone, 1e8, k=100
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for round in 1 2; do for v in $VARIANTS; do
  run 120 ab2_${v}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
done; done
