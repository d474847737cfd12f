#!/bin/bash
# Session 3: workgroup pairing of similar-extent groups (LSKNN_PAIR_WINDOW 0/16/64/256),
# 1e8 uniform, k=100, 2 rounds; GPU kernel tests with pairing on.
source scripts/gpu_check.sh
export TMPDIR=/tmp
for round in 1 2; do
  for w in 0 16 64 256; do
    run 150 s3pair_w${w}_$round.log env LSKNN_PAIR_WINDOW=$w python scripts/knn_only.py --points 1e8 --reps 3
  done
done
run 600 s3pair_tests.log env LSKNN_PAIR_WINDOW=64 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread
