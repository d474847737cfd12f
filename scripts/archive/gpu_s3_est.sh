#!/bin/bash
# Session 3: nearest group members kept for the per-lane first-range estimate
# (LSK_EST_M 4 / 6 / 8), 1e8 uniform, k=100, 2 interleaved rounds; 2e7 clustered check.
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for round in 1 2; do
  for v in em8 em6 em4; do
    run 150 s3e_${v}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
  done
done
