#!/bin/bash
# Radix-sort A/B (lib/exp variants s0..s4, scripts/build_variant.py): sort_bench at 1B
# (checks the sorted output) for each, alternating twice; then the sort GPU tests on s2.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for rep in 1 2; do
  for v in s0 s1 s2 s3 s4; do
    LSKNN_HIP_LIB=$X/liblsknn_hip_$v.so run 240 sort_${v}_$rep.log python -u scripts/sort_bench.py 1e9 || exit $?
    echo "$v $rep: $(grep -h 'sort check\|n=' gpurun_out/sort_${v}_$rep.log | tr '\n' ' ')"
  done
done
LSKNN_HIP_LIB=$X/liblsknn_hip_s2.so run 300 sort_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py || exit $?
tail -2 gpurun_out/sort_tests.log
