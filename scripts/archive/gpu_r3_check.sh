# stream tests, the driver's 1B bench, 1e8 stream, then PMC passes of the grid kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local t=$1 log=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run 300 chk_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stream.py tests/test_bench_cli.py -m gpu
run 500 chk_1b.log python -u bench.py --steps 20 --warmup 5
run 300 chk_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 3
bash scripts/gpu_pmc_r3.sh
