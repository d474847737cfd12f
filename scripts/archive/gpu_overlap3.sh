#!/bin/bash
# Tighter a-priori radius bound: distributed GPU tests + loopback halo sizes / timing.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 ov3_tests.log python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_kernels.py -v -x --timeout 300 --timeout-method thread
run 300 ov3_lb_on.log python scripts/loopback_phases.py 2e8 8 --nomarks
