#!/bin/bash
# Exact backstop over failure lists: waves per listed query (LSK_EXACT_LIST_WAVES 4 / 8 / 16)
# on mixed-scale 2e7 (192 failed queries at k=100), after the backstop tests per variant.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_DISTS=mixed_scale
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in base lw16 lw4 base lw16; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 200 lw_tests_$v.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "fail or exact or heavy" || exit 1
  grep -q " passed" gpurun_out/lw_tests_$v.log && ! grep -q "failed" gpurun_out/lw_tests_$v.log || exit 1
  LSKNN_HIP_LIB=$L run 200 lw_$v.log python -u scripts/dist_robustness.py 2e7 100 16 || exit 1
  echo "== $v"; grep -h "^{'dist'" gpurun_out/lw_$v.log
done
