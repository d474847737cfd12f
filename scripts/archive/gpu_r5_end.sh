#!/bin/bash
# PMC passes of the final grid kernel at 3e7, then the 8-rank per-rank replay at 1B.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
KERNS=sgpr TAG=_final PTS=3e7 bash scripts/gpu_r5_pmc.sh > gpurun_out/pmc_final.log 2>&1 || { echo "pmc failed"; exit 3; }
cat gpurun_out/pmc5_final/summary.txt
run 600 r5e_replay_1b_8.log python -u scripts/rank_replay.py 1e9 8 || exit $?
grep -h "SUMMARY" gpurun_out/r5e_replay_1b_8.log
