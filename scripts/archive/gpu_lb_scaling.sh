#!/bin/bash
# Kernel traces of the unordered pipeline emulated with P = 2, 4, 8 loopback ranks on one
# GPU (1B points, k=100): per-rank GPU kernel time (ranks serialize on one stream).
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
for P in 2 4 8; do
  run 500 lb${P}_trace.log rocprofv3 --kernel-trace -d $O/lb$P -o run --output-format csv -- python3 scripts/loopback_phases.py 1e9 $P
done
