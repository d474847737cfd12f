#!/bin/bash
# Session-3 checkpoint: full GPU suite, smoke, default bench (pipelined 1B), kernel stats
# of the default bench, forced RCCL 1e8 on both communicators (pipelined default).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 900 s3f_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 120 s3f_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 400 s3f_bench.log python bench.py --steps 20 --warmup 2
run 400 s3f_prof.log timeout -s KILL 380 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/s3f_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --verify 0
run 300 s3f_rccl_nccl.log env LSKNN_DIST_BACKEND=nccl MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
run 300 s3f_rccl_native.log env LSKNN_DIST_BACKEND=rccl MASTER_ADDR=127.0.0.1 MASTER_PORT=29572 python bench.py --force-dist --points 1e8 --steps 10 --warmup 2
