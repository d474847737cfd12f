#!/bin/bash
# knn_mfma occupancy probe: band lists in global memory (no LDS limit), MINW 3..6.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in ${VARIANTS:-g3 g4 g5 g6}; do
  run 200 r5f_$v.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/mfma_check.py --points 1e6 1e7 --k 100 --reps 2 --oracle 500
  run 200 r5f_${v}_big.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/mfma_check.py --points 1e8 --k 100 --reps 3 --only mfma
done
for v in ${VARIANTS:-g3 g4 g5 g6}; do echo "== $v"; grep -v amdgpu.ids gpurun_out/r5f_$v.log gpurun_out/r5f_${v}_big.log; done
