#!/bin/bash
# Sort tile size A/B on the 1B build pieces (scripts/sort_bench.py).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r5i_sort_base.log python scripts/sort_bench.py 1e9
for v in s24 s32; do
  run 300 r5i_sort_$v.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/sort_bench.py 1e9
done
for v in base s24 s32; do echo "== $v"; grep -v amdgpu.ids gpurun_out/r5i_sort_$v.log; done
