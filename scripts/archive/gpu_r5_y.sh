#!/bin/bash
# 8-rank per-rank replay at 1B with the two-stream local pass timings, then the MINW 6
# grid-kernel variant A/B at 1e8.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 600 r5y_replay_1b_8.log python -u scripts/rank_replay.py 1e9 8 || exit $?
grep -h "SUMMARY\|local_split" gpurun_out/r5y_replay_1b_8.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('SUMMARY'): print(l.strip()); continue
    r = json.loads(l); print(r['rank'], r['local_ms'], r['local_split'])
"
V=m6 bash scripts/gpu_r5_r.sh || exit $?
