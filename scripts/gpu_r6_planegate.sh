#!/bin/bash
# The FRAME_RADIUS_X gate: flat-frame tests, then the tilted plane at 2e7 (frame taken) and 2e8 (refused).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_DISTS=tilted_plane LSK_REPS=3
run 300 r6pg_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat_frame.py tests/test_gpu_graph.py || exit $?
grep -q " passed" gpurun_out/r6pg_tests.log && ! grep -q " failed" gpurun_out/r6pg_tests.log || { echo "STOP: tests failed"; exit 5; }
for n in 2e7 2e8; do
  run 300 r6pg_$n.log python -u scripts/dist_robustness.py $n 100 48 || exit $?
done
for f in gpurun_out/r6pg_2e*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f; done
