#!/bin/bash
# Exact backstop: GPU kernel tests + smoke + 1e8 kernel timing.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 900 r2_tests_kernels.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph.py -x -v --timeout 300 --timeout-method thread
run 180 r2_knn.log python scripts/knn_only.py --points 1e8 --reps 3 --impl rows
