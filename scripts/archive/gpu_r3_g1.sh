set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/g1_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/g1_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e7 --k 100 > gpurun_out/g1_ab_1e7.log 2>&1 && cat gpurun_out/g1_ab_1e7.log && \
timeout -k 10 300 python -u scripts/grid_ab.py --points 1e8 --k 100 > gpurun_out/g1_ab_1e8.log 2>&1 && cat gpurun_out/g1_ab_1e8.log
