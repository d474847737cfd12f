#!/bin/bash
# Kernel stats of the index build pieces at 1B (sort_bench) for sort variants s0 (HEAD form) and s3.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in s0 s3; do
  LSKNN_HIP_LIB=$X/liblsknn_hip_$v.so run 300 sortprof_$v.log rocprofv3 --kernel-trace --stats -d gpurun_out/sortprof_$v -o sp -- python3 -u scripts/sort_bench.py 1e9 || exit $?
done
for v in s0 s3; do echo "== $v"; f=$(find gpurun_out/sortprof_$v -name '*kernel_stats.csv' | head -1); head -12 "$f" | cut -d, -f1-5; done
