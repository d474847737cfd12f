#!/bin/bash
# Hardware queues A/B on the 1B stream: bench (8 by default) vs 4, and the SetStream probe
# at 8 queues (it ran at the box's 4 before: 887-892 ms per set).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r5n_bench_q8.log python bench.py --steps 10 --warmup 3 --verify 0
run 300 r5n_bench_q4.log env LSKNN_HW_QUEUES=4 python bench.py --steps 10 --warmup 3 --verify 0
run 300 r5n_probe_q8.log env GPU_MAX_HW_QUEUES=8 python -u scripts/stream_d2h_probe.py 1e9 8 copy copy
run 300 r5n_bench_q8b.log python bench.py --steps 10 --warmup 3 --verify 0
for f in r5n_bench_q8 r5n_bench_q4 r5n_bench_q8b; do grep -h '"metric"' gpurun_out/$f.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$f', r['ms_per_step'], r['value'], r['config']['hw_queues'], r['single_set_ms'])"; done
grep -v amdgpu.ids gpurun_out/r5n_probe_q8.log
