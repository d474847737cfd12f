# kernel trace + stats of the 1B stream bench (current kernels), per-set k-NN timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_s2 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --verify 0 > gpurun_out/prof_s2_bench.log 2>&1 || exit $?
tail -1 gpurun_out/prof_s2_bench.log | cut -c1-600
python3 scripts/timeline.py gpurun_out/prof_s2 knn_grid > gpurun_out/prof_s2_timeline.txt 2>&1
find gpurun_out/prof_s2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_s2_kernel_stats.csv
head -25 gpurun_out/prof_s2_kernel_stats.csv | cut -d, -f1-8
