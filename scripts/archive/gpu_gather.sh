#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 g_tests.log python -u -m pytest tests/test_gpu_kernels.py -k "gather3 or knn_uniform" -v -x --timeout 200 --timeout-method thread
run 400 g_prof.log timeout -s KILL 380 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/g_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1
