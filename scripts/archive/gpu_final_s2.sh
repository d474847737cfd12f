# end-of-session check: full GPU suite, smoke, the driver's 1B bench, the table configs,
# and a kernel-stats profile of the 1B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 900 fin_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu
grep -q " passed" gpurun_out/fin_tests.log && ! grep -q "failed" gpurun_out/fin_tests.log || exit 1
run 200 fin_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run 500 fin_bench_1b.log python -u bench.py --gpus 1 --steps 20 --warmup 5
run 300 fin_bench_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 3
run 200 fin_bench_1e7_k16.log python -u bench.py --points 1e7 --k 16 --steps 20 --warmup 3
run 200 fin_bench_1e6_k8.log python -u bench.py --points 1e6 --k 8 --steps 50 --warmup 5
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --verify 0 > gpurun_out/fin_prof.log 2>&1 || exit $?
