#!/bin/bash
# A/B: k-NN kernel alone for each variant library (lib/exp/liblsknn_hip_<v>.so), 1e8
# uniform points, interleaved twice; then the oracle kernel tests against variant $TESTV.
source scripts/gpu_check.sh
export TMPDIR=/tmp
for round in 1 2; do
  for v in $1; do
    run 120 ab_${v}_$round.log env LSKNN_HIP_LIB=$PWD/mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
  done
done
if [ -n "$TESTV" ]; then
  run 600 tests_$TESTV.log env LSKNN_HIP_LIB=$PWD/mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$TESTV.so python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py -q -x --timeout 300 --timeout-method thread
fi
