# round 4 p: defaults with 8 queues; build-ahead (next set's build beside the k-NN)
# re-measured now that streams no longer share queues
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
LSKNN_DIST_BACKEND=nccl run 300 fd_p.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_DIST_BACKEND=nccl LSKNN_BUILD_AHEAD=1 run 300 fd_p_ahead.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
run 300 s1e8_p.log python -u bench.py --points 1e8 --steps 20 --warmup 3
LSKNN_BUILD_AHEAD=1 run 300 s1e8_p_ahead.log python -u bench.py --points 1e8 --steps 20 --warmup 3
run 400 s1b_p.log python -u bench.py --steps 10 --warmup 3
LSKNN_BUILD_AHEAD=1 run 400 s1b_p_ahead.log python -u bench.py --steps 10 --warmup 3
