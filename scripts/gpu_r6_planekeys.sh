#!/bin/bash
# 2-D Morton keys for planes in their rotated frame (LSKNN_PLANE_KEYS=2d) vs the 3-D curve keys,
# the frame forced at every size (LSKNN_FRAME_RADIUS_X=0): tilted plane 2e7 / 2e8 / 5e8, k = 100, 48.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_DISTS=tilted_plane LSK_REPS=3 LSKNN_FRAME_RADIUS_X=0
run 300 r6pk_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat_frame.py || exit $?
grep -q " passed" gpurun_out/r6pk_tests.log && ! grep -q " failed" gpurun_out/r6pk_tests.log || { echo "STOP: tests failed"; exit 5; }
for n in 2e7 2e8 5e8; do for kk in 2d 3d; do
  run 300 r6pk_${n}_$kk.log env LSKNN_PLANE_KEYS=$kk python -u scripts/dist_robustness.py $n 100 48 || exit $?
done; done
for f in gpurun_out/r6pk_*e*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f; done
