#!/bin/bash
# Session 3: row queue capacity A/B (LSK_RCAP 32 default / 16 / 16 with 1-node flushes and
# fill 4), 1e8 uniform, k=100, 2 interleaved rounds.
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for round in 1 2; do
  for v in rc32 rc16 rc16p2; do
    run 150 s3r_${v}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
  done
done
