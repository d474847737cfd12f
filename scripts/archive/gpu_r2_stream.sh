#!/bin/bash
# Streamed redistribution: GPU tests, forced 1-rank RCCL bench, P=8 gloo rehearsal + trace.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 400 r2st_tests.log python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_gpu_multiprocess.py tests/test_bench_cli.py -v -x --timeout 200 --timeout-method thread
run 300 r2st_force_1e8.log python bench.py --points 1e8 --steps 3 --warmup 1 --force-dist
run 400 r2st_force_1b.log python bench.py --steps 3 --warmup 1 --force-dist
