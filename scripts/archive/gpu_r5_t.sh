#!/bin/bash
# Learned heavy-cell refinement in a stream: GPU stream tests + A/B on mixed-scale sets.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
true
run 500 r5t_ab.log python -u scripts/stream_heavy_ab.py 5e6 6 mixed_scale
grep -v "amdgpu.ids\|HW_QUEUES" gpurun_out/r5t_ab.log
