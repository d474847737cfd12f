set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b1_bench.log 2>&1; tail -1 gpurun_out/b1_bench.log | cut -c1-1500
