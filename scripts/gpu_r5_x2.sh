#!/bin/bash
# gpu_r5_x.sh (GPU suite + final benches) and the 8-rank per-rank replay at 1B.
source scripts/gpu_check.sh
bash scripts/gpu_r5_x.sh || exit $?
run 600 r5x_replay_1b_8.log python -u scripts/rank_replay.py 1e9 8 || exit $?
grep -h "SUMMARY" gpurun_out/r5x_replay_1b_8.log
