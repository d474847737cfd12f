#!/bin/bash
# Fused point gather in the sort's last pass (LSKNN_FUSED_GATHER) A/B: sort/gather GPU tests,
# build pieces at 1B, then the driver's 1B bench, alternating twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r6fg_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_grid.py || exit $?
for g in 1 0; do run 200 r6fg_sb_$g.log env LSKNN_FUSED_GATHER=$g python -u scripts/sort_bench.py 1e9 || exit $?; done
for r in 1 2; do for g in 1 0; do
  run 300 r6fg_bench_${g}_$r.log env LSKNN_FUSED_GATHER=$g python -u bench.py --steps 10 --warmup 3 || exit $?
done; done
grep -h "whole build" gpurun_out/r6fg_sb_*.log
for f in gpurun_out/r6fg_bench_*.log; do grep -h '"metric"' $f | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$f', r['value'], r['ms_per_step'], r['single_set_mpts'], r['detail']['phase_ms_max_over_ranks'], r['config'].get('sampled_exact'))"; done
