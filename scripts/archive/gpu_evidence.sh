#!/bin/bash
# Evidence round: PMC counters of the k-NN kernel, kernel-trace stats of the 1B bench,
# and the BASELINE.md table.
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
bash scripts/gpu_pmc_knn.sh || exit $?
run 600 prof_1b.log rocprofv3 --kernel-trace --stats -d $O/prof_1b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1
bash scripts/gpu_bench_table.sh
