# round 4 e: grid level sweep (k-NN kernel alone, uniform)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 200 lvl_1e7.log python -u scripts/grid_level_sweep.py 1e7 100
run 300 lvl_1e8.log python -u scripts/grid_level_sweep.py 1e8 100
run 500 lvl_1e9.log python -u scripts/grid_level_sweep.py 1e9 100 9 10
run 200 lvl_1e8_k16.log python -u scripts/grid_level_sweep.py 1e8 16
