#!/bin/bash
# 1B bench (current defaults) + kernel trace of the 8-rank loopback pipeline on 1B points.
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
run 600 bench_1b.log python bench.py --steps 3 --warmup 1 --phases
run 600 lb8_trace.log rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/lb8 -o run --output-format csv -- python3 scripts/loopback_phases.py 1e9 8
