#!/bin/bash
# Variant libraries ($V) : oracle check at 1e6 (k = 16, 100), the grid GPU tests with the
# variant loaded (unless NOTEST), then 1e8 k=100 timing against production, twice.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PTS=${PTS:-1e8}
for v in $V; do
  L=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so
  run 200 r6v_${v}_oracle.log env LSKNN_HIP_LIB=$L python scripts/knn_ab.py --points 1e6 --k 16 100 --reps 2 --oracle 2000 || exit $?
  grep -q "2000/2000" gpurun_out/r6v_${v}_oracle.log || { echo "STOP: $v oracle mismatch"; grep oracle gpurun_out/r6v_${v}_oracle.log; exit 1; }
  if [ -z "$NOTEST" ]; then
    run 400 r6v_${v}_tests.log env LSKNN_HIP_LIB=$L python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py || exit $?
  fi
done
for r in 1 2; do
  run 200 r6v_prod_$r.log python scripts/knn_ab.py --points $PTS --k 100 --reps 5 || exit $?
  for v in $V; do
    run 200 r6v_${v}_$r.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/knn_ab.py --points $PTS --k 100 --reps 5 || exit $?
  done
done
for f in gpurun_out/r6v_*_[12].log; do echo "$(basename $f): $(grep -h 'n=' $f)"; done
