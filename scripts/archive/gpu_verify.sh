#!/bin/bash
# Quick verification: GPU tests, smoke, k-NN kernel alone, 1B bench, rocprofv3 stats.
source scripts/gpu_check.sh
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
run 900 tests_gpu.log python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread --durations=8
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 120 knn_rows.log python scripts/knn_only.py --points 1e8 --reps 2 --impl rows
run 900 bench_1b.log python bench.py --steps 3 --warmup 1 --phases
run 300 prof_stats.log rocprofv3 --kernel-trace --stats -d $OUT/prof_stats -o run --output-format csv -- python3 bench.py --points 1e8 --steps 2 --warmup 1
