#!/bin/bash
# Round 2: graph-capturable refinement tests, slow-distribution diagnostics.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 400 r2r_tests.log python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_kernels.py -x -v -s --timeout 250 --timeout-method thread
run 300 r2r_slow.log python scripts/debug_slow_dists.py 2e7
