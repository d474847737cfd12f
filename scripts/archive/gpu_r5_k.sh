#!/bin/bash
# The default-backend tests (native RCCL, agreed fallback) + the forced-RCCL bench tests.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 600 r5k_tests.log python -u -m pytest tests/test_bench_cli.py tests/test_gpu_rccl.py tests/test_cli_apps.py -m gpu -x -v --timeout 200 --timeout-method thread
tail -15 gpurun_out/r5k_tests.log
