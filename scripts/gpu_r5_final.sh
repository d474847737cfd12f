#!/bin/bash
# Round-5 final check: the driver's bench command, the smoke, a 1e8 forced multi-rank
# stream on the default (native RCCL) communicator, and a kernel-trace profile.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run 300 r5f_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 600 r5f_bench_1b.log python bench.py --gpus 1 --steps 20 --warmup 5
run 300 r5f_fd_1e8.log python bench.py --force-dist --points 1e8 --steps 20 --warmup 3
run 300 r5f_1e8.log python bench.py --points 1e8 --steps 20 --warmup 3
O=$PWD/gpurun_out/r5f_trace
mkdir -p $O
run 400 r5f_trace.log timeout -s KILL 360 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --verify 0
python3 scripts/timeline.py $O knn_grid --gaps > gpurun_out/r5f_timeline.txt 2>&1 || true
f=$(find $O -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r5f_kernel_stats.csv
for f in r5f_bench_1b r5f_fd_1e8 r5f_1e8; do grep -h '"metric"' gpurun_out/$f.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$f', r['value'], r['ms_per_step'], r['single_set_mpts'], r['config']['comm_info'], r['config'].get('sampled_exact'))"; done
tail -1 gpurun_out/r5f_smoke.log; head -8 gpurun_out/r5f_timeline.txt
