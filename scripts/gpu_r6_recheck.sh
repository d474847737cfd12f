#!/bin/bash
# Round-6 re-check on a rebuilt tree: full GPU suite, smoke, the driver's bench command and
# every distribution at 2e7 (k=100, 16).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 600 rc_gpu_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ || exit $?
grep -q " passed" gpurun_out/rc_gpu_tests.log && ! grep -q " failed" gpurun_out/rc_gpu_tests.log || { echo "STOP: GPU tests failed"; exit 5; }
run 300 rc_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 600 rc_bench_1b.log python bench.py --gpus 1 --steps 20 --warmup 5
grep -h '"metric"' gpurun_out/rc_bench_1b.log | cut -c1-400
export LSK_DISTS=uniform,clustered,duplicates,planar,mixed_scale,tilted_plane,line
run 600 rc_robust.log python -u scripts/dist_robustness.py 2e7 100 16 || exit $?
grep -h "^{'dist'" gpurun_out/rc_robust.log
