#!/bin/bash
# Keyed streamed upload (single rank): tests, graph bench, kernel trace of the overlap.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 up_tests.log python -u -m pytest tests/test_gpu_distributed.py tests/test_bench_cli.py tests/test_gpu_graph.py -m gpu -v -x --timeout 300 --timeout-method thread
run 400 up_bench.log python bench.py --steps 10 --warmup 2
run 400 up_prof.log timeout -s KILL 380 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $PWD/gpurun_out/up_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1
