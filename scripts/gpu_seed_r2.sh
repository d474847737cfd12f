#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
for sd in 1 2 3; do
  run 150 seed_$sd.log python scripts/knn_only.py --points 1e8 --reps 3 --seed $sd
done
run 600 tests_def.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py tests/test_gpu_graph.py -q -x --timeout 300 --timeout-method thread
