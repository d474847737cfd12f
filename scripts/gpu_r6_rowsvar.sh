#!/bin/bash
# knn_rows tuning constants on the sets it serves (clustered, planar, mixed-scale; 2e7,
# k=100 / 16): library variants $VARIANTS (scripts/build_variant.py) vs production.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_DISTS=${LSK_DISTS:-clustered,planar,mixed_scale} LSK_REPS=3
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in base ${VARIANTS:-wpb1 wpb4} base; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 200 rk_$v.log python -u scripts/dist_robustness.py 2e7 100 16 || exit 1
  echo "== $v"; grep -h "^{'dist'" gpurun_out/rk_$v.log
done
