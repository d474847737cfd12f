set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_grid.py tests/test_stream.py tests/test_gpu_refalgo.py > gpurun_out/b3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/b3_tests.log; [ $rc -eq 0 ] || exit $rc
for d in 0 1; do timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 --direct-out $d > gpurun_out/b3_d$d.log 2>&1; echo "direct=$d"; tail -1 gpurun_out/b3_d$d.log | cut -c1-420; done
