#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 400 r2e_tests.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph.py -v -x --timeout 200 --timeout-method thread
run 300 r2e_slow.log python scripts/debug_slow_dists.py 2e7 mixed_scale
