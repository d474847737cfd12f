# round 4 ad: kernel trace + stats of the final 1B stream (per-set k-NN / build timeline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ad_trace -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --verify 0 > gpurun_out/ad_bench.log 2>&1
python3 scripts/timeline.py gpurun_out/ad_trace knn_grid --gaps > gpurun_out/ad_timeline.txt
find gpurun_out/ad_trace -name '*kernel_stats.csv' -exec cp {} gpurun_out/ad_kernel_stats.csv \;
