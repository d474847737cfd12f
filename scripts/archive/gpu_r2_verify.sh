#!/bin/bash
# Round 2: full GPU suite + smoke + 1e8 kernel timing + 1B bench.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 r2_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 120 r2_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 180 r2_knn.log python scripts/knn_only.py --points 1e8 --reps 3 --impl rows
run 400 r2_bench.log python bench.py --steps 5 --warmup 2
