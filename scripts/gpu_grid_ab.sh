set -o pipefail
cd $GRAFT_REPO_ROOT
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/gridab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gridab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 8 > gpurun_out/gridab_1e8.log 2>&1; grep -v "^build" gpurun_out/gridab_1e8.log
echo "== branchless"; LSKNN_HIP_LIB=$X/liblsknn_hip_bl.so timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 8 > gpurun_out/gridab_bl.log 2>&1; grep "grid\|bitwise" gpurun_out/gridab_bl.log
timeout -k 10 400 python -u scripts/grid_ab.py --points 1e9 --k 100 --levels 9 > gpurun_out/gridab_1b.log 2>&1; cat gpurun_out/gridab_1b.log
