#!/bin/bash
# Scheduler-strategy variants: knn_grid at 1e8 (gpu_r5_r.sh), then knn_rows on non-uniform
# data with the iterative-minreg library (gpu_r5_rows.sh).
source scripts/gpu_check.sh
V="imr iil imo imr7" bash scripts/gpu_r5_r.sh || exit $?
V="imr" bash scripts/gpu_r5_rows.sh || exit $?
