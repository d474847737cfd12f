set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/g10_tests.log 2>&1; rc=$?; tail -2 gpurun_out/g10_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/grid_build_cost.py 2e7 100 2>&1 | grep -v amdgpu
timeout -k 10 200 python -u scripts/grid_build_cost.py 1e8 100 2>&1 | grep -v amdgpu
LSKNN_GRID=auto timeout -k 10 400 python -u scripts/dist_robustness.py 2e7 100 16 > gpurun_out/g10_auto.log 2>&1; grep -v "^{" gpurun_out/g10_auto.log | grep -v amdgpu
