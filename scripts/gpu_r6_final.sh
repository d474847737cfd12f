#!/bin/bash
# Round-6 final check: the driver's bench command, the smoke, a 1e8 forced multi-rank
# stream on the default (native RCCL) communicator, and a kernel-trace profile.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r6f_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 600 r6f_bench_1b.log python bench.py --gpus 1 --steps 20 --warmup 5
run 300 r6f_fd_1e8.log python bench.py --force-dist --points 1e8 --steps 20 --warmup 3
run 300 r6f_1e8.log python bench.py --points 1e8 --steps 20 --warmup 3
O=$PWD/gpurun_out/r6f_trace
mkdir -p $O
run 400 r6f_trace.log timeout -s KILL 360 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --verify 0
python3 scripts/timeline.py $O knn_grid --gaps > gpurun_out/r6f_timeline.txt 2>&1 || true
f=$(find $O -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r6f_kernel_stats.csv
for f in r6f_bench_1b r6f_fd_1e8 r6f_1e8; do grep -h '"metric"' gpurun_out/$f.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$f', r['value'], r['ms_per_step'], r['single_set_mpts'], r['config']['comm_info'], r['config'].get('sampled_exact'))"; done
tail -1 gpurun_out/r6f_smoke.log; head -8 gpurun_out/r6f_timeline.txt
python3 - <<'PY' > gpurun_out/r6f_kernel_stats_summary.txt
import csv
rows = list(csv.DictReader(open("gpurun_out/r6f_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:70]:70s} calls {int(r["Calls"]):4d} avg {float(r["AverageNs"]) / 1e6:9.3f} ms  total {float(r["TotalDurationNs"]) / 1e6:9.2f} ms  {100 * float(r["TotalDurationNs"]) / tot:5.1f} %')
PY
head -6 gpurun_out/r6f_kernel_stats_summary.txt
