#!/bin/bash
# Kernel trace of the 1B build pieces (per-kernel times of the sort passes, gather, tree).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$PWD/gpurun_out/r5j
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/sort_bench.py 1e9 > $O/log.txt 2>&1 || exit 1
f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 $f | head -30
