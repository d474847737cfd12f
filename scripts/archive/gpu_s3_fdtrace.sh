#!/bin/bash
# Session 3: kernel + copy trace of the forced 1-rank RCCL pipelined bench at 1e8 (the
# per-rank size of an 8-GPU 1B run): where the non-k-NN time of a multi-rank step goes.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 400 s3f_trace.log timeout -s KILL 380 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $PWD/gpurun_out/s3f_trace -o run --output-format csv -- python3 bench.py --force-dist --points 1e8 --steps 4 --warmup 1 --verify 0
