set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e8 --k 100 --levels 7,8,9 > gpurun_out/g2_1e8.log 2>&1; cat gpurun_out/g2_1e8.log
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e7 --k 100 --levels 6,7,8 > gpurun_out/g2_1e7.log 2>&1; cat gpurun_out/g2_1e7.log
timeout -k 10 200 python -u scripts/grid_ab.py --points 1e7 --k 16 --levels 6,7,8 > gpurun_out/g2_1e7k16.log 2>&1; cat gpurun_out/g2_1e7k16.log
