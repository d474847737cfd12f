#!/bin/bash
# Overlapped halo exchange: GPU tests (loopback + 1-rank RCCL), loopback P=8 phases with
# and without overlap, kernel trace of the overlapped loopback run (no phase syncs).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 ov_tests.log python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_gpu_multiprocess.py tests/test_bench_cli.py -m gpu -v -x --timeout 300 --timeout-method thread
run 300 ov_lb_on.log python scripts/loopback_phases.py 2e8 8 --nomarks
run 300 ov_lb_off.log env LSKNN_OVERLAP_HALO=0 python scripts/loopback_phases.py 2e8 8 --nomarks
run 300 ov_trace.log timeout -s KILL 280 rocprofv3 --kernel-trace -d $PWD/gpurun_out/ov_trace -o run --output-format csv -- python3 scripts/loopback_phases.py 2e8 8 --nomarks
python scripts/halo_overlap_trace.py gpurun_out/ov_trace > gpurun_out/ov_overlap.txt 2>&1
