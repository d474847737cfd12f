#!/bin/bash
# Rotated index frame for flat data (LSKNN_FLAT_FRAME): GPU tests, then every distribution
# at 2e7 (k=100, 16) with the frame on and off, alternating twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ -z "$NOTEST" ]; then
  run 400 r6ff_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat_frame.py tests/test_gpu_kernels.py || exit $?
  grep -q " passed" gpurun_out/r6ff_tests.log && ! grep -q " failed" gpurun_out/r6ff_tests.log || { echo "STOP: tests failed"; exit 5; }
fi
export LSK_DISTS=${LSK_DISTS:-tilted_plane,line,planar,clustered,duplicates,mixed_scale}
for r in 1 2; do for f in 1 0 e; do
  if [ $f = e ]; then ENVS="LSKNN_FLAT_FRAME=1 LSKNN_FRAME_EARLY=1"; else ENVS="LSKNN_FLAT_FRAME=$f"; fi
  run 300 r6ff_${f}_$r.log env $ENVS python -u scripts/dist_robustness.py 2e7 100 16 || exit $?
done; done
for f in gpurun_out/r6ff_[01e]_*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f | python3 -c "
import sys, ast
print('  ' + '  '.join(f\"{d['dist']}/{d['k']} {d['Mpts_s']} ({d['exact']})\" for d in map(ast.literal_eval, sys.stdin)))"; done
