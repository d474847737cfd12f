# round 4 c: exact-backstop box counting (mixed-scale), staged gate read (stream), short
# boundary lists (per-rank replay); tests first, then the measurements
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 600 t_c.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_grid.py tests/test_gpu_distributed.py tests/test_stream.py
run 300 mixed_probe.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixed -o run --output-format csv -- python3 -u scripts/mixed_probe.py 20000000 100 16
LSK_DISTS=mixed_scale,clustered,duplicates,planar run 400 robust_2e7.log python -u scripts/dist_robustness.py 20000000 100 16
run 400 s_1b.log python -u bench.py --steps 10 --warmup 3
run 400 replay_1b_8.log python -u scripts/rank_replay.py 1e9 8
run 300 s_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 3
export LSKNN_DIST_BACKEND=nccl
run 300 fd_1e8.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
