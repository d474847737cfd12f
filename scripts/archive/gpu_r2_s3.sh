#!/bin/bash
# Session-3 re-verification of the restored tree: GPU suite, smoke, default 1B bench.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 800 s3_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 120 s3_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 400 s3_bench.log python bench.py --steps 10 --warmup 2
