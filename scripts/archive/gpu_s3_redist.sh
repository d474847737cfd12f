#!/bin/bash
# Session 3: next set's redistribution under the current set's k-NN (SetStream, several
# ranks): bench/stream/forced-dist GPU tests, forced 1-rank RCCL 1e8 on both
# communicators, 8 gloo ranks on one GPU (2e8) rehearsal.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3x_tests.log python -u -m pytest tests/test_stream.py tests/test_bench_cli.py tests/test_forced_dist.py tests/test_gpu_multiprocess.py -m gpu -x -v --timeout 300 --timeout-method thread
run 300 s3x_fd_nccl.log env MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
run 300 s3x_fd_rccl.log env LSKNN_DIST_BACKEND=rccl MASTER_ADDR=127.0.0.1 MASTER_PORT=29592 python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
run 600 s3x_g8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29593 bench.py --gpus 8 --points 2e8 --steps 3 --warmup 1
