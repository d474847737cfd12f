#!/bin/bash
# Multi-rank readiness: the distributed GPU tests, then the per-rank
# replay of the unordered pipeline at 1B over 2 / 4 / 8 ranks and 1e8 over 2 / 4 / 8 ranks
# (every run checks its outputs bitwise against one rank).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ -z "$NOTEST" ]; then
  run 500 r6r_dist_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_stream.py -m gpu || exit $?
  grep -q " passed" gpurun_out/r6r_dist_tests.log && ! grep -q " failed" gpurun_out/r6r_dist_tests.log || { echo "STOP: tests failed"; exit 5; }
fi
for spec in ${SPECS:-1e9:8 1e9:4 1e9:2 1e8:8 1e8:4 1e8:2}; do
  n=${spec%%:*}; p=${spec##*:}
  run 400 r6r_replay_${n}_${p}.log python -u scripts/rank_replay.py $n $p || exit $?
done
grep -h "SUMMARY" gpurun_out/r6r_replay_*.log
