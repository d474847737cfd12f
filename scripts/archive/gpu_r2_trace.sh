#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 r2tr.log timeout -s KILL 280 rocprofv3 --kernel-trace --memory-copy-trace -d $PWD/gpurun_out/r2tr -o run --output-format csv -- python3 bench.py --points 2e8 --steps 2 --warmup 1 --force-dist --verify 0
python scripts/trace_overlap.py gpurun_out/r2tr > gpurun_out/r2tr_overlap.txt 2>&1
