#!/bin/bash
# Native RCCL communicator: 1-rank forced tests (ROCm 2.27 and torch 2.26 RCCL), bench.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 rn_tests.log python -u -m pytest tests/test_gpu_rccl.py tests/test_bench_cli.py -m gpu -v -s -x --timeout 300 --timeout-method thread
run 300 rn_bench.log env LSKNN_DIST_BACKEND=rccl python bench.py --force-dist --points 1e8 --steps 3 --warmup 1
run 300 rn_bench_nccl.log env LSKNN_DIST_BACKEND=nccl python bench.py --force-dist --points 1e8 --steps 3 --warmup 1
