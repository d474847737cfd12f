#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
for sd in 0 1 2; do
  run 150 seed_$sd.log python scripts/knn_only.py --points 1e8 --reps 3 --seed $sd
done
