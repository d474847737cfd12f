#!/bin/bash
# Stream heavy-cell policy: tests, mixed-scale stream (learned), uniform 1B bench (no regression).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 600 r5u_tests.log python -u -m pytest tests/test_stream.py -m gpu -x -q --timeout 200 --timeout-method thread
run 300 r5u_ab.log env LSK_MODES=learned python -u scripts/stream_heavy_ab.py 5e6 6 mixed_scale
run 300 r5u_bench.log python bench.py --steps 10 --warmup 3
tail -2 gpurun_out/r5u_tests.log; grep -v "amdgpu.ids\|HW_QUEUES" gpurun_out/r5u_ab.log | tail -3
grep -h '"metric"' gpurun_out/r5u_bench.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench', r['value'], r['ms_per_step'], r['single_set_mpts'], r['config']['heavy_cells_unrefined'], r['config'].get('sampled_exact'))"
