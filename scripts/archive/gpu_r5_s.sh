#!/bin/bash
# knn_mfma with the wave-queue appends (variant library) vs production sgpr: bitwise + time.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=${V:-q1}
L=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$V.so
run 200 r5s_${V}_small.log env LSKNN_HIP_LIB=$L python scripts/mfma_check.py --points 1e6 --k 8 16 100 --oracle 1000 --reps 2
run 300 r5s_${V}_big.log env LSKNN_HIP_LIB=$L python scripts/mfma_check.py --points 1e7 1e8 --k 100 --reps 3
grep -hv "amdgpu.ids\|HW_QUEUES" gpurun_out/r5s_${V}_small.log gpurun_out/r5s_${V}_big.log
