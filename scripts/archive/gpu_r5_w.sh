#!/bin/bash
# Batch-8 grid kernel variant: grid GPU tests on the variant, then 1B bench A/B.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_b8.so
run 600 r5w_tests.log env LSKNN_HIP_LIB=$L python -u -m pytest tests/test_gpu_grid.py -m gpu -x -q --timeout 200 --timeout-method thread
run 300 r5w_bench_b8.log env LSKNN_HIP_LIB=$L python bench.py --steps 10 --warmup 3
run 300 r5w_bench_base.log python bench.py --steps 10 --warmup 3
run 300 r5w_bench_b8b.log env LSKNN_HIP_LIB=$L python bench.py --steps 10 --warmup 3
tail -2 gpurun_out/r5w_tests.log
for f in r5w_bench_b8 r5w_bench_base r5w_bench_b8b; do grep -h '"metric"' gpurun_out/$f.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$f', r['value'], r['ms_per_step'], r['config'].get('sampled_exact'))"; done
