#!/bin/bash
# Remaining BASELINE table configs with the round-6 build: 1M k=8, 10M k=16, prePartitioned 1e8.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 t6_1m_k8.log python -u bench.py --points 1e6 --k 8 --steps 20 --warmup 5 || exit $?
run 300 t6_10m_k16.log python -u bench.py --points 1e7 --k 16 --steps 20 --warmup 5 || exit $?
run 300 t6_100m_pre.log python -u bench.py --points 1e8 --steps 10 --warmup 3 --variant prepartitioned || exit $?
for f in t6_1m_k8 t6_10m_k16 t6_100m_pre; do grep -h '"metric"' gpurun_out/$f.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$f', r['value'], r['ms_per_step'], r.get('single_set_mpts'), r['config'].get('sampled_exact'))"; done
