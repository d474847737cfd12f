set -o pipefail
cd $GRAFT_REPO_ROOT
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/g6_tests.log 2>&1; rc=$?; tail -2 gpurun_out/g6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7,8 > gpurun_out/g6_1e8.log 2>&1; grep -v "^build" gpurun_out/g6_1e8.log
for v in top8 top10; do echo "== $v"; LSKNN_HIP_LIB=$X/liblsknn_hip_$v.so timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7,8 > gpurun_out/g6_$v.log 2>&1; grep "grid-L\|bitwise" gpurun_out/g6_$v.log; done
LSKNN_HIP_LIB=$X/liblsknn_hip_gprof.so timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7,8 --reps 1 > gpurun_out/g6_prof.log 2>&1; grep -A1 "grid-L" gpurun_out/g6_prof.log
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e7 --k 16 --levels 6,7 > gpurun_out/g6_1e7k16.log 2>&1; grep -v "^build" gpurun_out/g6_1e7k16.log
