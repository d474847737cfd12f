# round 4 m: hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4): with more
# streams than queues, unrelated streams serialise in one queue
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
export LSKNN_DIST_BACKEND=nccl
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q run 300 fd_q$q.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
done
unset LSKNN_DIST_BACKEND
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q run 300 s1e8_q$q.log python -u bench.py --points 1e8 --steps 20 --warmup 3
done
GPU_MAX_HW_QUEUES=8 run 400 s1b_q8.log python -u bench.py --steps 10 --warmup 3
