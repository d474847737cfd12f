#!/bin/bash
# Session 3: multi-rank pipelined bench with the result D2H on its own stream under the
# next step: bench GPU tests, forced 1-rank RCCL 1e8 (x2), 1B single-rank default.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3d_tests.log python -u -m pytest tests/test_bench_cli.py -m gpu -x -v --timeout 300 --timeout-method thread
run 300 s3d_fd_1.log python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
run 300 s3d_fd_2.log python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
run 400 s3d_1b.log python bench.py --steps 10 --warmup 2
