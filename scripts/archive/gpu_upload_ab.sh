#!/bin/bash
# Single-rank keyed upload: chunk size A/B on the 1B bench (0 = one copy, keys after).
source scripts/gpu_check.sh
export TMPDIR=/tmp
for c in 0 134217728 67108864 0 134217728 67108864; do
  run 400 upab_$c.log env LSKNN_UPLOAD_CHUNK=$c python bench.py --steps 8 --warmup 2 --verify 0
  grep -h metric gpurun_out/upab_$c.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('chunk $c', r['ms_per_step'])" >> gpurun_out/upab_summary.txt
done
