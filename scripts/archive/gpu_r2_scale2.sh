#!/bin/bash
# Round 2: chunked RCCL messages — tests, forced-RCCL bench at 1e8 and 1B.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 r2s_tests.log python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 250 --timeout-method thread
run 300 r2s_bench_force_1e8.log python bench.py --points 1e8 --steps 3 --warmup 1 --force-dist
run 400 r2s_bench_force_1b.log python bench.py --steps 3 --warmup 1 --force-dist
