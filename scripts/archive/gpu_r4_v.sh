# round 4 v: network band selection only for waves with a band of > 8 values (small k keeps
# the heap); k=16 / k=8 / k=100 checks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 300 v_tests.log python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_grid.py
run 300 v_1e7_k16.log python -u bench.py --points 1e7 --k 16 --steps 20 --warmup 5
run 300 v_1e6_k8.log python -u bench.py --points 1e6 --k 8 --steps 20 --warmup 5
run 300 v_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 5
run 200 v_knn.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
