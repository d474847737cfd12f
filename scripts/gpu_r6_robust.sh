#!/bin/bash
# Throughput + sampled exactness on every synthetic distribution at 2e7 points, k=100 and 16
# (production library).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_DISTS=uniform,clustered,duplicates,planar,mixed_scale,tilted_plane,line
run 600 r6_robust_final.log python -u scripts/dist_robustness.py 2e7 100 16 || exit $?
grep -h "^{'dist'" gpurun_out/r6_robust_final.log
