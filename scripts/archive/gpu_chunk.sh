#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
for c in 33554432 16777216 8388608 33554432; do
  run 300 ch_$c.log env LSKNN_STREAM_CHUNK=$c python bench.py --force-dist --points 1e8 --steps 5 --warmup 1
done
