#!/bin/bash
# Session 3: single-rank pipelined bench with the next set's index build on a
# high-priority side stream (default) vs copy-only prefetch (LSKNN_PIPE_BUILD=0).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3o_tests.log python -u -m pytest tests/test_bench_cli.py -m gpu -x -v --timeout 300 --timeout-method thread
for round in 1 2; do
  run 400 s3o_build_$round.log python bench.py --steps 10 --warmup 2 --verify 64
  run 400 s3o_copy_$round.log env LSKNN_PIPE_BUILD=0 python bench.py --steps 10 --warmup 2 --verify 64
done
