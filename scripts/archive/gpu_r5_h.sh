#!/bin/bash
# GPU suite after the default-backend change, then the non-uniform grid probe.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 900 r5h_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 500 r5h_nonuni.log python scripts/grid_nonuniform.py 2e7 8 9 10
tail -3 gpurun_out/r5h_tests.log; grep -v amdgpu.ids gpurun_out/r5h_nonuni.log
run 500 r5h_replay.log python -u scripts/rank_replay.py 1e9 8
grep -v amdgpu.ids gpurun_out/r5h_replay.log | tail -4
