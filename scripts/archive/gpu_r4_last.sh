# round 4, last check of the committed tree: GPU suite, smoke, the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 1100 last_tests.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
run 300 last_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run 500 last_bench_1b.log python -u bench.py
