#!/bin/bash
# High-priority RCCL streams: 1-rank RCCL tests + forced-RCCL bench kernel trace (halo
# kernels and RCCL kernels under the k-NN).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 ov2_tests.log python -u -m pytest tests/test_gpu_rccl.py tests/test_bench_cli.py -m gpu -v -x --timeout 300 --timeout-method thread
run 300 ov2_trace.log timeout -s KILL 280 rocprofv3 --kernel-trace -d $PWD/gpurun_out/ov2_trace -o run --output-format csv -- python3 bench.py --force-dist --points 1e8 --steps 2 --warmup 1
python scripts/halo_overlap_trace.py gpurun_out/ov2_trace > gpurun_out/ov2_overlap.txt 2>&1
