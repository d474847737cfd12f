set -o pipefail
cd $GRAFT_REPO_ROOT
export LSKNN_HIP_LIB=$PWD/mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_gprof.so
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7 --reps 1 > gpurun_out/g4_1e8.log 2>&1; cat gpurun_out/g4_1e8.log
