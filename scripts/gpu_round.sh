#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
run 120 build.log python mpi_cuda_largescaleknn_amd/_build.py
run 900 t13.log python -m pytest tests/ -q -m gpu -x --durations=5
run 120 knn_rows.log python scripts/knn_only.py --points 1e8 --reps 2 --impl rows
run 120 knn_wave.log python scripts/knn_only.py --points 1e8 --reps 2 --impl wave
run 600 bench1b.log python bench.py --steps 3 --warmup 1 --phases
run 300 prof13.log rocprofv3 --kernel-trace --stats -d $OUT/prof13 -o run --output-format csv -- python3 bench.py --points 1e8 --steps 2 --warmup 1
