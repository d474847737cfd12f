# round 4 final check, part 2: table configs, per-rank replay, robustness
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 300 fin_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 5
run 300 fin_1e7_k16.log python -u bench.py --points 1e7 --k 16 --steps 20 --warmup 5
run 300 fin_1e6_k8.log python -u bench.py --points 1e6 --k 8 --steps 20 --warmup 5
run 300 fin_pre_1e8.log python -u bench.py --variant prepartitioned --points 1e8 --steps 20 --warmup 5
LSKNN_DIST_BACKEND=nccl run 300 fin_fd_1e8.log python -u bench.py --force-dist --points 1e8 --steps 20 --warmup 5
run 400 fin_replay_1b_8.log python -u scripts/rank_replay.py 1e9 8
LSK_DISTS=uniform,clustered,duplicates,planar,mixed_scale run 400 fin_robust_2e7.log python -u scripts/dist_robustness.py 20000000 100 16
