#!/bin/bash
# Non-uniform data on the production path: build vs k-NN, kernel counters.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 400 r5l_nonuni_stats.log python scripts/nonuniform_stats.py 2e7 100
grep -v amdgpu.ids gpurun_out/r5l_nonuni_stats.log
