#!/bin/bash
# build_variant.sh NAME "-DFOO=1 ..." : kernel library with knn_rows.hip built with extra
# defines, at mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_NAME.so (tuning experiments)
set -e
cd "$(dirname "$0")/.."
L=mpi_cuda_largescaleknn_amd/lib
mkdir -p $L/exp
python mpi_cuda_largescaleknn_amd/_build.py > /dev/null
objs=$(ls $L/obj/*.o | grep -v knn_rows)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -mllvm -disable-promote-alloca-to-vector --offload-arch=gfx950 $2 \
  -c mpi_cuda_largescaleknn_amd/csrc/hip/knn_rows.hip -o $L/exp/knn_rows_$1.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "error|VGPRs:|Occupancy|LDS S|Spill" | sort | uniq
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/exp/liblsknn_hip_$1.so $objs $L/exp/knn_rows_$1.o
