#!/bin/bash
# Session 3: next set's index build on a CU-masked stream beside the current k-NN
# (LSKNN_BUILD_CUS = 0 / 16 / 32 / 64 of 256 CUs), 1B pipelined bench; stream GPU tests.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 s3c_tests.log python -u -m pytest tests/test_stream.py -m gpu -x -v --timeout 200 --timeout-method thread
for round in 1 2; do
  for c in 0 16 32 64; do
    run 400 s3c_cus${c}_$round.log env LSKNN_BUILD_CUS=$c python bench.py --steps 8 --warmup 1 --verify 32
  done
done
