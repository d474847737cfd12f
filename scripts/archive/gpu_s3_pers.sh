#!/bin/bash
# Session 3: persistent grid-stride k-NN waves (pers1) vs the same looped kernel on a
# one-group-per-wave grid (pers0) vs the previous kernel (base2), 1e8 uniform, k=100;
# then the GPU kernel tests on pers1 and an occupancy pass.
source scripts/gpu_check.sh
export TMPDIR=/tmp
L=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for round in 1 2; do
  for v in base2 pers0 pers1; do
    run 150 s3pe_${v}_$round.log env LSKNN_HIP_LIB=$L/liblsknn_hip_$v.so python scripts/knn_only.py --points 1e8 --reps 3
  done
done
run 600 s3pe_tests.log env LSKNN_HIP_LIB=$L/liblsknn_hip_pers1.so python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py tests/test_gpu_graph.py -v -x --timeout 120 --timeout-method thread
run 120 s3pe_pmc.log env LSKNN_HIP_LIB=$L/liblsknn_hip_pers1.so timeout -s KILL 110 rocprofv3 --pmc OccupancyPercent -d $PWD/gpurun_out/s3pe_pmc -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
