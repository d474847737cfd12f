set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --verify 0 > gpurun_out/trace_bench.log 2>&1
tail -1 gpurun_out/trace_bench.log | cut -c1-300
python3 scripts/timeline.py gpurun_out/trace knn_grid
