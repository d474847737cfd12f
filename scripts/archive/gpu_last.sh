# last check of the committed tree: full GPU suite, smoke, the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 900 last_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu
grep -q " passed" gpurun_out/last_tests.log && ! grep -q "failed" gpurun_out/last_tests.log || exit 1
run 200 last_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run 500 last_bench.log python -u bench.py --gpus 1 --steps 20 --warmup 5
