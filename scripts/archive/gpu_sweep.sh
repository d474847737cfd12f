#!/bin/bash
# Macro / parameter sweep of the k-NN kernel (1e8 uniform, k=100), interleaved twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for round in 1 2; do
  for v in base exec0 tb12 tb20 cg8; do
    run 120 sw_${v}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
  done
  for sd in 1 3; do
    run 120 sw_seed${sd}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_base.so python scripts/knn_only.py --points 1e8 --reps 3 --seed $sd
  done
done
