# round 4 b: changed GPU tests, then per-rank replay at 1B / 8, 1B bench with kernel stats,
# forced 1-rank stream, robustness
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 1000 t_changed.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_grid.py tests/test_gpu_distributed.py tests/test_gpu_kernels.py tests/test_stream.py tests/test_gpu_rccl.py
run 400 replay_1b_8.log python -u scripts/rank_replay.py 1e9 8
run 500 s_1b_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1b -o run --output-format csv -- python3 -u bench.py --steps 6 --warmup 2 --verify 64
run 400 s_1b.log python -u bench.py --steps 10 --warmup 3
LSK_DISTS=mixed_scale,clustered run 400 robust_2e7.log python -u scripts/dist_robustness.py 20000000 100 16
export LSKNN_DIST_BACKEND=nccl
run 300 fd_1e8.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
unset LSKNN_DIST_BACKEND
run 300 mixed_probe.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixed -o run --output-format csv -- python3 -u scripts/mixed_probe.py 20000000 100 16
