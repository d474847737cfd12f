#!/bin/bash
# Non-uniform data on the grid kernel at forced levels.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 400 r5g_nonuni.log python scripts/grid_nonuniform.py 2e7 7 8 9
grep -v amdgpu.ids gpurun_out/r5g_nonuni.log
