# round 4 n: with 8 hardware queues: redistribution under / after the k-NN, full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
export LSKNN_DIST_BACKEND=nccl
LSKNN_REDIST_UNDER_KNN=0 run 300 fd_n_after.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_REDIST_UNDER_KNN=1 run 300 fd_n_under.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_REDIST_UNDER_KNN=0 run 300 fd_n_after2.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_REDIST_UNDER_KNN=1 run 300 fd_n_under2.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
unset LSKNN_DIST_BACKEND
run 1100 t_full.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
