#!/bin/bash
# Lines sorted along their axis in their own frame (LSKNN_LINE_KEYS) vs 3-D curve keys: flat-frame
# tests, then the line at 2e7 and 2e8 (k = 100, 16), on / off.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_REPS=3 LSK_DISTS=line
run 300 r6lk_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat_frame.py || exit $?
grep -q " passed" gpurun_out/r6lk_tests.log && ! grep -q " failed" gpurun_out/r6lk_tests.log || { echo "STOP: tests failed"; exit 5; }
for n in 2e7 2e8; do for f in 1 0; do
  run 300 r6lk_${n}_$f.log env LSKNN_LINE_KEYS=$f python -u scripts/dist_robustness.py $n 100 16 || exit $?
done; done
for f in gpurun_out/r6lk_2e*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f; done
