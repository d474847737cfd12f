#!/bin/bash
# Session-3 last GPU call: stream/bench tests, driver bench command, and a kernel trace of
# the forced 1-rank multi-rank stream (next set's redistribution under the k-NN).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 s3l_tests.log python -u -m pytest tests/test_stream.py tests/test_bench_cli.py -m gpu -x -v --timeout 300 --timeout-method thread
run 600 s3l_bench.log python3 bench.py --gpus 1 --steps 20 --warmup 5
run 400 s3l_trace.log env MASTER_ADDR=127.0.0.1 MASTER_PORT=29601 timeout -s KILL 380 rocprofv3 --kernel-trace --memory-copy-trace -d $PWD/gpurun_out/s3l_trace -o run --output-format csv -- python3 bench.py --force-dist --points 1e8 --steps 4 --warmup 1 --verify 0
