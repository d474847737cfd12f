set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/g3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7,8 > gpurun_out/g3_1e8.log 2>&1; cat gpurun_out/g3_1e8.log
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e7 --k 16 --levels 6,7 > gpurun_out/g3_1e7k16.log 2>&1; cat gpurun_out/g3_1e7k16.log
