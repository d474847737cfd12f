# round 4 b: changed GPU tests, then benches (forced 1-rank stream, 1e8 stream,
# prePartitioned 1e8 graph + stream, 1B stream), per-rank replay at 1B / 8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 1000 t_changed.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grid.py tests/test_gpu_graph.py tests/test_stream.py tests/test_gpu_rccl.py tests/test_gpu_distributed.py tests/test_gpu_kernels.py
export LSKNN_DIST_BACKEND=nccl
run 300 fd_1e8.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
unset LSKNN_DIST_BACKEND
run 200 s_1e8.log python -u bench.py --points 1e8 --steps 10 --warmup 3
run 200 pre_1e8_graph.log python -u bench.py --points 1e8 --steps 10 --warmup 3 --variant prepartitioned --pipeline 0
run 200 pre_1e8_stream.log python -u bench.py --points 1e8 --steps 10 --warmup 3 --variant prepartitioned
run 400 s_1b.log python -u bench.py --steps 10 --warmup 3
run 400 replay_1b_8.log python -u scripts/rank_replay.py 1e9 8
LSK_DISTS=mixed_scale,uniform,clustered run 400 robust_2e7.log python -u scripts/dist_robustness.py 20000000 100 16
