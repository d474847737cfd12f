#!/bin/bash
# End-of-round checkpoint: full GPU suite, smoke, default 1B bench, kernel stats, forced
# RCCL 1e8 bench on both communicators, robustness table.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 800 fin_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 120 fin_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 400 fin_bench.log python bench.py --steps 10 --warmup 2
run 400 fin_prof.log timeout -s KILL 380 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/fin_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1
run 300 fin_rccl_nccl.log env LSKNN_DIST_BACKEND=nccl python bench.py --force-dist --points 1e8 --steps 5 --warmup 1
run 300 fin_rccl_native.log env LSKNN_DIST_BACKEND=rccl python bench.py --force-dist --points 1e8 --steps 5 --warmup 1
run 400 fin_rob.log python scripts/dist_robustness.py
