#!/bin/bash
# Heavy-run threshold of the key refinement (LSKNN_HEAVY_RUN): 4096 / 256 / 64 on clustered,
# mixed-scale and uniform data at 2e7, k = 100 / 16, alternating twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_REPS=3 LSK_DISTS=clustered,mixed_scale,uniform
for r in 1 2; do for h in 4096 256 64; do
  run 300 r6hr_${h}_$r.log env LSKNN_HEAVY_RUN=$h python -u scripts/dist_robustness.py 2e7 100 16 || exit $?
done; done
for f in gpurun_out/r6hr_*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f | python3 -c "
import sys, ast
print('  ' + '  '.join(f\"{d['dist']}/{d['k']} {d['Mpts_s']} ({d['exact']})\" for d in map(ast.literal_eval, sys.stdin)))"; done
