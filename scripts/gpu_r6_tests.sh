#!/bin/bash
# Round-6 end check: full GPU suite, then gpu_r6_final.sh (driver bench, smoke, forced RCCL,
# 1e8, kernel trace).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 600 r6x_gpu_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ || exit $?
grep -q " passed" gpurun_out/r6x_gpu_tests.log && ! grep -q " failed" gpurun_out/r6x_gpu_tests.log || { echo "STOP: GPU tests failed"; exit 5; }
