#!/bin/bash
# 8 ranks on ONE GPU over gloo (host-staged collectives) with the pipelined default:
# rehearsal of the driver's 8-GPU launch (not an xGMI/RCCL measurement).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3g8_2e8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --points 2e8 --steps 2 --warmup 1
run 900 s3g8_1b.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 8 --steps 2 --warmup 1
