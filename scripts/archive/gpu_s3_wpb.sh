#!/bin/bash
# Session 3: GPU suite on the 2-waves-per-block k-NN kernel (default build) incl. the
# MPI two-ranks-on-one-GPU test, then the 1B bench A/B of 4 vs 2 waves per block.
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
run 800 s3w_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
for round in 1 2; do
  run 300 s3w_bench_wpb4_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_wpb4.so python bench.py --steps 5 --warmup 1 --verify 0
  run 300 s3w_bench_wpb2_$round.log python bench.py --steps 5 --warmup 1 --verify 0
done
