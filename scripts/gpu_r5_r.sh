#!/bin/bash
# knn_grid A/B: variant libraries ($V, space-separated names of scripts/build_variant.py
# builds) vs production, 1e8 k=100, alternating twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=${V:-ev}
for r in 1 2; do
  run 200 r5r_base_$r.log python scripts/knn_ab.py --points 1e8 --k 100 --reps 5 || exit $?
  for v in $V; do
    run 200 r5r_${v}_$r.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/knn_ab.py --points 1e8 --k 100 --reps 5 || exit $?
  done
done
for f in gpurun_out/r5r_*.log; do echo "$(basename $f): $(grep -h 'sgpr:' $f)"; done
