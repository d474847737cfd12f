# round 4 k: per-set upload events (the copy stream shares a hardware queue with the result
# copy): forced 1-rank RCCL stream with 1 / 4 launches, host timeline, streams, tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 600 t_k.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stream.py tests/test_gpu_rccl.py tests/test_forced_dist.py tests/test_bench_cli.py
export LSKNN_DIST_BACKEND=nccl
LSKNN_KNN_CHUNKS=1 run 300 dbg_hook3.log python -u scripts/debug_hook.py 1e8
LSKNN_KNN_CHUNKS=1 run 300 fd_k_c1.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_KNN_CHUNKS=4 run 300 fd_k_c4.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
LSKNN_KNN_CHUNKS=4 run 300 fd_k_c4_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fd4 -o run --output-format csv -- python3 -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
unset LSKNN_DIST_BACKEND
run 400 s_1b_k.log python -u bench.py --steps 10 --warmup 3
