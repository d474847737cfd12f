#!/bin/bash
# Quick check after a kernel/pipeline change: GPU tests, smoke, 1e8 kernel, 1B bench.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 tests_gpu.log python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 120 knn_rows.log python scripts/knn_only.py --points 1e8 --reps 2 --impl rows
run 600 bench_1b.log python bench.py --steps 3 --warmup 1 --phases
