#!/bin/bash
# Exact backstop: expansion step (LSK_EXACT_STEP 3 / 6) x waves per listed query (8 / 16)
# on mixed-scale 2e7 (failure lists) and uniform 2e6 at k=300 (whole-set exact kernel),
# after the backstop tests per variant.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in base lw16 s6w16 s6w8 base s6w16; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 200 es_tests_$v.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_flat_frame.py -k "fail or exact or heavy or frame" || exit 1
  grep -q " passed" gpurun_out/es_tests_$v.log && ! grep -q "failed" gpurun_out/es_tests_$v.log || exit 1
  LSK_DISTS=mixed_scale LSKNN_HIP_LIB=$L run 200 es_$v.log python -u scripts/dist_robustness.py 2e7 100 16 || exit 1
  LSK_DISTS=uniform,clustered LSKNN_HIP_LIB=$L run 200 es_big_$v.log python -u scripts/dist_robustness.py 2e6 300 || exit 1
  echo "== $v"; grep -h "^{'dist'" gpurun_out/es_$v.log gpurun_out/es_big_$v.log
done
