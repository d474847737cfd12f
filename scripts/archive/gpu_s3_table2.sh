#!/bin/bash
# Session 3: bench tests after the 1e7-point threshold of the stream default; 1M k=8
# (single set, HIP graph) and the driver's 1B command.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3u_tests.log python -u -m pytest tests/test_bench_cli.py -m gpu -x -v --timeout 300 --timeout-method thread
run 300 s3t_1m_k8_graph.log python bench.py --points 1e6 --k 8 --steps 20 --warmup 5
run 600 s3u_bench.log python3 bench.py --gpus 1 --steps 20 --warmup 5
