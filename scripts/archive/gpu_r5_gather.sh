#!/bin/bash
# gather3 tile A/B (LSK_G3PER rows per lane: 4 production, 8, 16) via sort_bench at 1B, alternating twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for r in 1 2; do
  run 240 gat_base_$r.log python -u scripts/sort_bench.py 1e9 || exit $?
  for v in g8 g16; do
    LSKNN_HIP_LIB=$X/liblsknn_hip_$v.so run 240 gat_${v}_$r.log python -u scripts/sort_bench.py 1e9 || exit $?
  done
done
for f in gpurun_out/gat_*.log; do echo "$(basename $f): $(grep -h 'sort check\|n=' $f | tr '\n' ' ')"; done
