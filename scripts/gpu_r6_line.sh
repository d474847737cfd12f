#!/bin/bash
# Lines in their principal frame with 1-D keys (LSKNN_LINE_FRAME): flat-frame GPU tests, then
# the line distributions at 2e7 (k=100, 16) with the line frame on and off, alternating twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r6ln_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat_frame.py || exit $?
grep -q " passed" gpurun_out/r6ln_tests.log && ! grep -q " failed" gpurun_out/r6ln_tests.log || { echo "STOP: tests failed"; exit 5; }
export LSK_DISTS=${LSK_DISTS:-line,tilted_plane}
for r in 1 2; do for f in 1 0; do
  run 300 r6ln_${f}_$r.log env LSKNN_LINE_FRAME=$f python -u scripts/dist_robustness.py 2e7 100 16 || exit $?
done; done
for f in gpurun_out/r6ln_[01]_*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f | python3 -c "
import sys, ast
print('  ' + '  '.join(f\"{d['dist']}/{d['k']} {d['Mpts_s']} ({d['exact']})\" for d in map(ast.literal_eval, sys.stdin)))"; done
