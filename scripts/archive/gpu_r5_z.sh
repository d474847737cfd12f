#!/bin/bash
# MINW 5 grid-kernel variant A/B at 1e8 against the default (6), then the 8-rank per-rank
# replay at 1B with the default.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=m5 bash scripts/gpu_r5_r.sh || exit $?
run 600 r5z_replay_1b_8.log python -u scripts/rank_replay.py 1e9 8 || exit $?
grep -h "SUMMARY" gpurun_out/r5z_replay_1b_8.log
