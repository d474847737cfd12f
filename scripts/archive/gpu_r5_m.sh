#!/bin/bash
# Dimension-aware first-pass estimate of the rows kernel: non-uniform stats + robustness
# (exactness) + the rows/grid GPU tests.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 400 r5m_nonuni_stats.log python scripts/nonuniform_stats.py 2e7 100
run 600 r5m_robust.log env LSK_REPS=3 LSK_DISTS=uniform,clustered,duplicates,planar,mixed_scale,tilted_plane,line python scripts/dist_robustness.py 2e7 100 16
run 900 r5m_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -v amdgpu.ids gpurun_out/r5m_nonuni_stats.log | grep -v counters; grep -v amdgpu.ids gpurun_out/r5m_robust.log; tail -2 gpurun_out/r5m_tests.log
run 400 r5m_d2h.log python -u scripts/stream_d2h_probe.py 1e9 8 copy nocopy copy
grep -v amdgpu.ids gpurun_out/r5m_d2h.log
