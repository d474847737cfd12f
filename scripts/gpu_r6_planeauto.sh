#!/bin/bash
# Plane frame with auto keys (2-D Morton above PLANE_2D_MIN): flat-frame tests; 2e8 tilted and
# axis-aligned planes, k = 100 / 16, frame (FRAME_MIN_K=1: also k = 16) vs own frame; 2e7 defaults.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_REPS=3
run 300 r6pa_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat_frame.py || exit $?
grep -q " passed" gpurun_out/r6pa_tests.log && ! grep -q " failed" gpurun_out/r6pa_tests.log || { echo "STOP: tests failed"; exit 5; }
export LSK_DISTS=tilted_plane,planar
run 300 r6pa_2e8_f1.log env LSKNN_FRAME_MIN_K=1 python -u scripts/dist_robustness.py 2e8 100 16 || exit $?
run 300 r6pa_2e8_f0.log env LSKNN_FLAT_FRAME=0 python -u scripts/dist_robustness.py 2e8 100 16 || exit $?
run 300 r6pa_2e7_def.log python -u scripts/dist_robustness.py 2e7 100 16 || exit $?
for f in gpurun_out/r6pa_2e*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f; done
