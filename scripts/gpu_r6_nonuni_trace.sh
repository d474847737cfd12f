#!/bin/bash
# Kernel trace of the non-uniform robustness sets (2e7, k=100): where the time goes per
# distribution (k-NN kernel, exact backstop, build).
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for d in ${DISTS:-planar tilted_plane line clustered}; do
  O=$PWD/gpurun_out/r6nt_$d
  mkdir -p $O
  run 300 r6nt_$d.log env LSK_DISTS=$d timeout -s KILL 250 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 scripts/dist_robustness.py 2e7 100 || exit $?
  f=$(find $O -name "*kernel_stats.csv" | head -1)
  echo "== $d"; python3 -c "
import csv
rows = list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(f'  {r[\"Name\"][:60]:60s} calls {int(r[\"Calls\"]):4d} avg {float(r[\"AverageNs\"]) / 1e6:8.3f} ms total {float(r[\"TotalDurationNs\"]) / 1e6:8.2f} ms')
"
done
