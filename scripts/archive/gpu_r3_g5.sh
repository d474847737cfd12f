set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/g5_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7 > gpurun_out/g5_1e8.log 2>&1; cat gpurun_out/g5_1e8.log
LSKNN_HIP_LIB=$PWD/mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_gprof.so timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7 --reps 1 > gpurun_out/g5_prof.log 2>&1; grep -A1 "grid" gpurun_out/g5_prof.log
