#!/bin/bash
# knn_mfma variant check: bitwise vs knn_grid (sgpr) + oracle samples, then 1e8 timing.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-d}
run 200 r5${T}_small.log python scripts/mfma_check.py --points 1e6 --k 8 16 100 --oracle 1000 --reps 2
run 300 r5${T}_big.log python scripts/mfma_check.py --points 1e7 1e8 --k 100 --reps 3
cat gpurun_out/r5${T}_small.log gpurun_out/r5${T}_big.log | grep -v amdgpu.ids
