#!/bin/bash
# Result copy on a narrow grid (K.copy_out) vs the runtime's blit, 1B stream.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r5q_unit.log python -u -m pytest tests/test_gpu_stream_copy.py -x -q --timeout 120 --timeout-method thread
run 400 r5q_probe.log python -u scripts/stream_d2h_probe.py 1e9 8 copy kcopy
run 400 r5q_probe8.log env LSKNN_COPY_OUT_BLOCKS=8 python -u scripts/stream_d2h_probe.py 1e9 8 kcopy
run 400 r5q_probe32.log env LSKNN_COPY_OUT_BLOCKS=32 python -u scripts/stream_d2h_probe.py 1e9 8 kcopy
run 300 r5q_bench_k.log env LSKNN_COPY_OUT=1 python bench.py --steps 10 --warmup 3
run 300 r5q_bench_0.log env LSKNN_COPY_OUT=0 python bench.py --steps 10 --warmup 3
grep -h "copy run" gpurun_out/r5q_probe*.log
for f in r5q_bench_k r5q_bench_0; do grep -h '"metric"' gpurun_out/$f.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$f', r['value'], r['ms_per_step'], r['single_set_mpts'], r['config'].get('sampled_exact'))"; done
tail -2 gpurun_out/r5q_unit.log
