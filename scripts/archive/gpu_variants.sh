#!/bin/bash
# A/B of kernel variants built by build_variant.sh (lib/exp/liblsknn_hip_<name>.so) on the
# k-NN kernel alone: gpu_variants.sh "<name> <name> ..." [points] [extra knn_only args]
source scripts/gpu_check.sh
export TMPDIR=/tmp
P=${2:-1e8}
for v in $1; do
  run 120 var_$v.log env LSKNN_HIP_LIB=$PWD/mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/knn_only.py --points $P --reps 3 $3
done
