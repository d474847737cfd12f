#!/bin/bash
# Histogram-resolution variants ($V, lib/exp) against production at ${PTS} uniform points
# and k in ${KS}: kernel time (median of 3) and the output hash (bit-identical check).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PTS=${PTS:-1e9}
KS=${KS:-100}
run 300 r6w_prod.log python scripts/knn_ab.py --points $PTS --k $KS --reps 3 || exit $?
for v in $V; do
  run 300 r6w_$v.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/knn_ab.py --points $PTS --k $KS --reps 3 || exit $?
done
for f in gpurun_out/r6w_*.log; do echo "$(basename $f):"; grep -h "n=" $f | cut -c1-200; done
