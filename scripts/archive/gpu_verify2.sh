#!/bin/bash
# tests + 1B bench + kernel trace of the 8-rank loopback pipeline (1B points)
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
run 600 tests_gpu.log python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread
run 600 bench_1b.log python bench.py --steps 3 --warmup 1 --phases
run 600 lb8_trace.log rocprofv3 --kernel-trace --stats -d $O/lb8 -o run --output-format csv -- python3 scripts/loopback_phases.py 1e9 8
python - > $O/lb8_kernels.txt <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/lb8/run_kernel_stats.csv")))
for r in rows[:40]:
    print(f"{float(r['TotalDurationNs'])/1e6:10.1f} ms {int(r['Calls']):6d}  {r['Name'][:110]}")
PY
