# round 4, first look: forced 1-rank RCCL stream (1e8) kernel trace, single-rank 1e8
# stream, grid kernel counters at 1e8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
export LSKNN_DIST_BACKEND=nccl
run 300 fd_1e8.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
run 300 fd_1e8_trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/fd_trace -o fd -- python3 -u bench.py --force-dist --points 1e8 --steps 6 --warmup 2 --graph 0
unset LSKNN_DIST_BACKEND
run 200 s_1e8.log python -u bench.py --points 1e8 --steps 10 --warmup 3
run 200 knn_1e8.log python -u scripts/knn_only.py --points 1e8 --grid 1 --reps 3
python scripts/timeline.py gpurun_out/fd_trace knn_ > gpurun_out/fd_timeline.txt 2>&1 || true
