#!/bin/bash
# Session 3: next set's redistribution issued right after the k-NN launch (before the
# halo exchange) on a high-priority stream: tests, forced 1-rank RCCL 1e8 on both
# communicators, trace, 8 gloo ranks on one GPU (2e8).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3y_tests.log python -u -m pytest tests/test_stream.py tests/test_bench_cli.py tests/test_forced_dist.py tests/test_gpu_multiprocess.py tests/test_gpu_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread
run 300 s3y_fd_nccl.log env MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
run 300 s3y_fd_rccl.log env LSKNN_DIST_BACKEND=rccl MASTER_ADDR=127.0.0.1 MASTER_PORT=29612 python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
run 400 s3y_trace.log env MASTER_ADDR=127.0.0.1 MASTER_PORT=29613 timeout -s KILL 380 rocprofv3 --kernel-trace -d $PWD/gpurun_out/s3y_trace -o run --output-format csv -- python3 bench.py --force-dist --points 1e8 --steps 4 --warmup 1 --verify 0
run 600 s3y_g8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 8 --points 2e8 --steps 3 --warmup 1
