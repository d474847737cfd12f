# A/B of kernel library variants (scripts/build_variant.py): grid tests on each, then the
# 1e8 k-NN pass (knn_only, 3 reps) base vs variants. VARIANTS="a b ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in $VARIANTS; do
  LSKNN_HIP_LIB=$X/liblsknn_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/vt_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/vt_$v.log; exit 1; }
  echo "== $v tests: $(tail -1 gpurun_out/vt_$v.log)"
done
N=${N:-1e8} VARIANTS="$VARIANTS" bash scripts/gpu_grid_variants.sh
