#!/bin/bash
# Round 2: RCCL 1-rank tests, bench contract tests, forced-RCCL bench, P=8 gloo rehearsal.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 r2s_tests.log python -u -m pytest tests/test_gpu_rccl.py tests/test_bench_cli.py -x -v --timeout 250 --timeout-method thread
run 300 r2s_bench_force_1e8.log python bench.py --points 1e8 --steps 3 --warmup 1 --force-dist
run 400 r2s_bench_1b.log python bench.py --steps 3 --warmup 1
run 600 r2s_bench_gloo8_1e8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --points 1e8 --steps 2 --warmup 1
