#!/bin/bash
# knn_rows scheduler variants on non-uniform data, then the 8-rank per-rank replay at 1B.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="rimo rdef" bash scripts/gpu_r5_rows.sh || exit $?
run 600 r5v_replay_1b_8.log python -u scripts/rank_replay.py 1e9 8 || exit $?
grep -h "SUMMARY" gpurun_out/r5v_replay_1b_8.log
