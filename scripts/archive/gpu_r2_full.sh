#!/bin/bash
# Round 2 checkpoint: full GPU suite, smoke, default 1B bench, kernel-trace stats of the bench.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 r2f_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 120 r2f_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 400 r2f_bench.log python bench.py --steps 10 --warmup 2
run 400 r2f_prof.log timeout -s KILL 380 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/r2f_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1
