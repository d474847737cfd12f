#!/bin/bash
# Round 5: GPU tests after the stream/bench changes; 1B PRE_KEYS A/B; 1B single-set
# UPLOAD_CHUNK A/B (8 queues); forced one-rank 1e8 torch-RCCL vs native-RCCL A/B.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
[ "$PART" = 2 ] || run 900 r5c_tests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
if [ "$PART" != 2 ]; then for v in 1 0; do
  run 300 r5c_prekeys_$v.log env LSKNN_PRE_KEYS=$v python bench.py --steps 10 --warmup 3 --verify 0
done; fi
[ "$PART" = 1 ] && exit 0
for c in 67108864 0; do
  run 300 r5c_upchunk_$c.log env LSKNN_UPLOAD_CHUNK=$c python bench.py --steps 4 --warmup 2 --verify 0
done
i=0; for b in nccl rccl nccl rccl; do i=$((i+1))
  run 200 r5c_dist_${b}_$i.log env LSKNN_DIST_BACKEND=$b python bench.py --force-dist --points 1e8 --steps 20 --warmup 3 --verify 0
done
grep -h '"metric"' gpurun_out/r5c_*.log > gpurun_out/r5c_json.txt
