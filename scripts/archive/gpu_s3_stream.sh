#!/bin/bash
# Session 3: SetStream (parallel/stream.py) refactor of the pipelined bench: stream and
# bench GPU tests, 1B default bench, forced 1-rank RCCL 1e8.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3s_tests.log python -u -m pytest tests/test_stream.py tests/test_bench_cli.py -m gpu -x -v --timeout 300 --timeout-method thread
run 400 s3s_bench.log python bench.py --steps 10 --warmup 2
run 300 s3s_fd.log env MASTER_ADDR=127.0.0.1 MASTER_PORT=29581 python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
