#!/bin/bash
# Standard GPU verification round: build, all GPU tests, smoke, kernel A/B, benches, profile.
source scripts/gpu_check.sh
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
run 120 build.log python mpi_cuda_largescaleknn_amd/_build.py
run 900 tests_gpu.log python -m pytest tests/ -q -m gpu -x --durations=5
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 120 knn_rows.log python scripts/knn_only.py --points 1e8 --reps 2 --impl rows
run 300 bench_100m.log python bench.py --points 1e8 --steps 3 --warmup 1 --phases
run 900 bench_1b.log python bench.py --steps 3 --warmup 1 --phases
run 300 prof_stats.log rocprofv3 --kernel-trace --stats -d $OUT/prof_stats -o run --output-format csv -- python3 bench.py --points 1e8 --steps 2 --warmup 1
run 900 lb8_1b.log python scripts/loopback_phases.py 1e9 8
