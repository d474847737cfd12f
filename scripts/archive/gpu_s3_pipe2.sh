#!/bin/bash
# Session 3: pipelined bench GPU tests (incl. 2 ranks on one GPU) + a kernel/copy trace
# of the 1B pipelined bench (H2D of the next set under the k-NN).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3q_tests.log python -u -m pytest tests/test_bench_cli.py -m gpu -x -v --timeout 300 --timeout-method thread
run 400 s3q_trace.log timeout -s KILL 380 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $PWD/gpurun_out/s3q_trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --verify 0
