#!/bin/bash
# Full GPU suite + smoke on the current tree.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r5v_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 1000 r5v_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r5v_smoke.log; tail -2 gpurun_out/r5v_tests.log
