# re-entry check: full GPU suite, smoke, the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 900 resume_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu
run 200 resume_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run 500 resume_bench.log python -u bench.py --gpus 1 --steps 20 --warmup 5
