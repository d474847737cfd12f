#!/bin/bash
# Session 3: k-NN kernel scheduler flags A/B (base3 = current flags; f1 + AMDGPU RP
# trackers; f2 + no unclustered high-RP reschedule), 1e8 uniform, k=100, 2 rounds.
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for round in 1 2; do
  for v in base3 f1 f2; do
    run 150 s3fl_${v}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
  done
done
