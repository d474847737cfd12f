#!/bin/bash
# A/B of kernel variants (lib/exp/liblsknn_hip_<v>.so) on 1e8 uniform points, k=100,
# interleaved rounds; optional test run on one variant (TESTV, verbose so a hang names
# its test).
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
if [ -n "$TESTV" ]; then
  run 600 tests_$TESTV.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$TESTV.so python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py tests/test_gpu_graph.py -v -x --timeout 120 --timeout-method thread
fi
for round in 1 2; do
  for v in $VARIANTS; do
    run 150 ab_${v}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points ${POINTS:-1e8} --reps 3
  done
done
for v in $PROFV; do
  run 200 prof_$v.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points ${POINTS:-1e8} --reps 1
done
