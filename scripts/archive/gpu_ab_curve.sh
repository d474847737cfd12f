#!/bin/bash
# A/B of the sort curve (Morton vs Hilbert): GPU tests, k-NN kernel alone, 1B bench.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 tests_gpu.log python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread
run 120 knn_morton.log env LSKNN_CURVE=morton python scripts/knn_only.py --points 1e8 --reps 2
run 120 knn_hilbert.log python scripts/knn_only.py --points 1e8 --reps 2
run 120 bound_hilbert.log python scripts/bound_experiment.py
run 900 bench_1b.log python bench.py --steps 3 --warmup 1 --phases
run 900 lb8_1b.log python scripts/loopback_phases.py 1e9 8
