#!/bin/bash
# knn_grid A/B (variant library vs production), 1e8 k=100, alternating.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=${V:-ev}
for r in 1 2; do
  run 200 r5r_base_$r.log python scripts/mfma_check.py --points 1e8 --k 100 --reps 5 --only sgpr
  run 200 r5r_${V}_$r.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$V.so python scripts/mfma_check.py --points 1e8 --k 100 --reps 5 --only sgpr
done
grep -h "sgpr:" gpurun_out/r5r_*.log
