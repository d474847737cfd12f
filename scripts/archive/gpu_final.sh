#!/bin/bash
# Round-end style verification: GPU suite, smoke, default bench (1B, k=100, HIP graph),
# kernel-trace stats of the graph-mode step at 1e8.
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
run 900 tests_gpu.log python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 600 bench_default.log python bench.py
run 300 prof_graph.log rocprofv3 --kernel-trace --stats -d $O/prof_graph -o run --output-format csv -- python3 bench.py --points 1e8 --steps 3 --warmup 1
