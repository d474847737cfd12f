#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for n in 6e4 1e5 1e6 1e7 1e8; do
  run 150 profsz_$n.log env LSKNN_HIP_LIB=$L/liblsknn_hip_profbf2.so python scripts/knn_only.py --points $n --reps 1
done
