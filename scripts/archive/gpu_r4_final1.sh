# round 4 final check, part 1: GPU suite, smoke, the driver's bench command, table configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 1100 fin_tests.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
run 300 fin_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run 500 fin_bench_1b.log python -u bench.py --gpus 1 --steps 20 --warmup 5
