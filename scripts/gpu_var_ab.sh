# k-NN pass of library variants ($VARIANTS, scripts/build_variant.py) at 1e8 against the
# default, after the grid tests on each variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 200 var_tests_$v.log python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_grid.py
  grep -q " passed" gpurun_out/var_tests_$v.log && ! grep -q "failed" gpurun_out/var_tests_$v.log || exit 1
  LSKNN_HIP_LIB=$L run 300 var_knn_$v.log python -u scripts/knn_only.py --points ${N:-1e8} --reps 3 --grid 1
done
