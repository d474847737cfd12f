# the driver's bench command (1B, k=100, stream of sets) + tests that guard it
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_grid.py tests/test_stream.py > gpurun_out/bench_tests.log 2>&1; rc=$?; tail -2 gpurun_out/bench_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench_1b.log 2>&1; tail -1 gpurun_out/bench_1b.log | cut -c1-1500
