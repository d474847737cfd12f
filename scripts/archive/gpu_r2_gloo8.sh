#!/bin/bash
# 8 ranks on ONE GPU over gloo (host-staged collectives): rehearsal of the 8-GPU bench
# launch at the headline size (not a measurement of xGMI/RCCL performance).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 900 r2_gloo8_1b.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 1 --warmup 1
