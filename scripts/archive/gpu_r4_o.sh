# round 4 o: 8 hardware queues effective in bench.py: redistribution after / under the k-NN;
# 1B and 1e8 streams
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
export LSKNN_DIST_BACKEND=nccl
LSKNN_REDIST_UNDER_KNN=0 run 300 fd_o_after.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_REDIST_UNDER_KNN=1 run 300 fd_o_under.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_REDIST_UNDER_KNN=0 run 300 fd_o_after2.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_REDIST_UNDER_KNN=1 run 300 fd_o_under2.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
unset LSKNN_DIST_BACKEND
run 300 s1e8_o.log python -u bench.py --points 1e8 --steps 20 --warmup 3
run 400 s1b_o.log python -u bench.py --steps 10 --warmup 3
