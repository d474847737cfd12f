# wrap-up: the bench CLI GPU tests (kernel names in the JSON), then PMC + trace of the
# final kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 600 wrap_benchcli.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_cli.py -m gpu
grep -q " passed" gpurun_out/wrap_benchcli.log && ! grep -q "failed" gpurun_out/wrap_benchcli.log || exit 1
bash scripts/gpu_pmc_final.sh
