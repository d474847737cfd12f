#!/bin/bash
# knn_rows histogram-resolution A/B ($V variants of scripts/build_variant.py vs production) on
# non-uniform 2e7-point sets, k=100 (scripts/dist_robustness.py), alternating twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_DISTS=${LSK_DISTS:-clustered,planar,tilted_plane,mixed_scale,line}
for r in 1 2; do
  run 300 r6w_base_$r.log python scripts/dist_robustness.py 2e7 100 || exit $?
  for v in $V; do
    run 300 r6w_${v}_$r.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/dist_robustness.py 2e7 100 || exit $?
  done
done
for f in gpurun_out/r6w_*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f | python3 -c "
import sys, ast
print('  ' + '  '.join(f\"{d['dist']} {d['Mpts_s']} ({d['exact']})\" for d in map(ast.literal_eval, sys.stdin)))"; done
