#!/bin/bash
# 8 processes on one GPU over gloo (host-staged): launch rehearsal with the round-2 final
# pipeline (streamed chunks, overlapped halo, grouped return, agreed collective forms).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 g8b.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --points 1e8 --steps 2 --warmup 1
