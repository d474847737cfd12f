#!/bin/bash
# Grouped result return: distributed GPU tests, forced-RCCL 1e8 bench (grouped return into
# pinned host memory), multiprocess gloo test.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 rt_tests.log python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_multiprocess.py tests/test_bench_cli.py tests/test_gpu_rccl.py -v -x --timeout 300 --timeout-method thread
run 300 rt_bench.log python bench.py --force-dist --points 1e8 --steps 3 --warmup 1
