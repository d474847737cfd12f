# build-ahead A/B: stream tests, then the 1B stream bench with the index build on the side
# stream (default) vs between the k-NN launches, then the 2e7 robustness table (best of 3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local t=$1 log=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 gpurun_out/$log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
run 300 ahead_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stream.py tests/test_gpu_grid.py tests/test_bench_cli.py -m gpu
LSKNN_BUILD_AHEAD=1 run 400 ahead_1b_on.log python -u bench.py --steps 10 --warmup 2
LSKNN_BUILD_AHEAD=0 run 400 ahead_1b_off.log python -u bench.py --steps 10 --warmup 2
LSKNN_BUILD_AHEAD=1 run 300 ahead_1e8_on.log python -u bench.py --points 1e8 --steps 20 --warmup 3
LSKNN_BUILD_AHEAD=0 run 300 ahead_1e8_off.log python -u bench.py --points 1e8 --steps 20 --warmup 3
LSKNN_BUILD_AHEAD=1 run 300 ahead_1e8_fd_on.log python -u bench.py --points 1e8 --steps 20 --warmup 3 --force-dist
LSKNN_BUILD_AHEAD=0 run 300 ahead_1e8_fd_off.log python -u bench.py --points 1e8 --steps 20 --warmup 3 --force-dist
LSKNN_GRID=off run 400 robust_off.log python -u scripts/dist_robustness.py 20000000 100 16
LSKNN_GRID=auto run 400 robust_auto.log python -u scripts/dist_robustness.py 20000000 100 16
