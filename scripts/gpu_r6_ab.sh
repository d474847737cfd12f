#!/bin/bash
# Round 6 knn_grid A/B: grid GPU tests on the production library, then variant libraries
# ($V: scripts/build_variant.py names; "base" = the library before the change) against
# production at 1e8 uniform, k = 100, alternating twice; outputs compared by their hash.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=${V:-base}
PTS=${PTS:-1e8}
if [ -z "$NOTEST" ]; then
  run 300 r6_grid_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grid.py || exit $?
  grep -q " passed" gpurun_out/r6_grid_tests.log && ! grep -q " failed" gpurun_out/r6_grid_tests.log || { echo "STOP: grid tests failed"; exit 1; }
  run 200 r6_oracle.log python scripts/knn_ab.py --points 1e6 --k 16 100 --reps 1 --oracle 2000 || exit $?
fi
for r in 1 2; do
  run 200 r6ab_prod_$r.log python scripts/knn_ab.py --points $PTS --k 100 --reps 5 || exit $?
  for v in $V; do
    run 200 r6ab_${v}_$r.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/knn_ab.py --points $PTS --k 100 --reps 5 || exit $?
  done
done
for f in gpurun_out/r6ab_*.log; do echo "$(basename $f): $(grep -h 'n=' $f)"; done
