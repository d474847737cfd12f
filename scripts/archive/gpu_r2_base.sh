#!/bin/bash
# Round-2 baseline: k-NN kernel stats at 1e8 (current kernel), 1B bench with phases.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 180 r2base_knn.log python scripts/knn_only.py --points 1e8 --reps 3 --impl rows
run 300 r2base_bench1e8.log python bench.py --points 1e8 --steps 3 --warmup 1 --phases --stats
