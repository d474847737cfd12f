# pair-layout (packed fp32) grid kernel: grid tests, A/B vs the AoS variant at 1e8, the
# driver's 1B bench, then the full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
run 300 pairs_gridtests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_grid.py
grep -q " passed" gpurun_out/pairs_gridtests.log && ! grep -q "failed" gpurun_out/pairs_gridtests.log || exit 1
for v in base aos pairhist branchless; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 300 pairs_knn_$v.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
run 500 pairs_bench.log python -u bench.py --gpus 1 --steps 20 --warmup 5
run 900 pairs_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu
run 200 pairs_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
