#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r5o_probe.log python -u scripts/stream_d2h_probe.py 1e9 10 copy
run 300 r5o_bench.log python bench.py --steps 10 --warmup 3 --verify 0
grep -v amdgpu.ids gpurun_out/r5o_probe.log; grep -h '"metric"' gpurun_out/r5o_bench.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench', r['ms_per_step'], r['value'])"
