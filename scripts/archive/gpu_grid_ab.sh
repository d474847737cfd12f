# grid tests, then grid (auto level + extra levels) vs tree k-NN A/B at 1e8 (+ cycle profile)
set -o pipefail
cd $GRAFT_REPO_ROOT
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid.py > gpurun_out/gridab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gridab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7,8,9 > gpurun_out/gridab_1e8.log 2>&1; grep -v "^build" gpurun_out/gridab_1e8.log
if [ -f $X/liblsknn_hip_gprof.so ]; then LSKNN_HIP_LIB=$X/liblsknn_hip_gprof.so timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 8 --reps 1 > gpurun_out/gridab_prof.log 2>&1; grep -A1 "^\[grid" gpurun_out/gridab_prof.log; fi
if [ -n "$AB_1B" ]; then timeout -k 10 400 python -u scripts/grid_ab.py --points 1e9 --k 100 --levels 9 > gpurun_out/gridab_1b.log 2>&1; grep -v "^build" gpurun_out/gridab_1b.log; fi
