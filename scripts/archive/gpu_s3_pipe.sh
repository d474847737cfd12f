#!/bin/bash
# Session 3: pipelined bench (two alternating sets, next upload under the k-NN):
# bench GPU tests, 1B pipelined vs not, forced 1-rank RCCL 1e8 streamed vs pipelined.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3p_tests.log python -u -m pytest tests/test_bench_cli.py -m gpu -x -v --timeout 300 --timeout-method thread
run 400 s3p_bench_pipe.log python bench.py --steps 10 --warmup 2
run 400 s3p_bench_nopipe.log python bench.py --steps 10 --warmup 2 --pipeline 0
run 300 s3p_fd_stream.log python bench.py --force-dist --points 1e8 --steps 5 --warmup 1 --pipeline 0
run 300 s3p_fd_pipe.log python bench.py --force-dist --points 1e8 --steps 5 --warmup 1 --pipeline 1
