set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stream.py tests/test_bench_cli.py > gpurun_out/b2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/b2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b2_bench.log 2>&1; tail -1 gpurun_out/b2_bench.log | cut -c1-1200
