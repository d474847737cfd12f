#!/bin/bash
# Crowded-bin pass abort: tests on the new default, non-uniform timings, uniform A/B.
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
run 400 crowd_tests.log env LSKNN_HIP_LIB=$L/liblsknn_hip_crowd16.so python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph.py -v -x --timeout 200 --timeout-method thread
for v in crowd16 crowd64; do
  run 300 crowd_slow_$v.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/debug_slow_dists.py 2e7 mixed_scale clustered
done
for v in ${AB:-}; do
  run 150 crowd_ab_${v}.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
done
