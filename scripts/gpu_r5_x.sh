#!/bin/bash
# Final round-5 check (driver bench, smoke, forced RCCL, 1e8, kernel trace), then the
# MINW 6 grid-kernel variant A/B at 1e8.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash scripts/gpu_r5_final.sh || exit $?
V=m6 bash scripts/gpu_r5_r.sh || exit $?
for f in gpurun_out/r5r_base_1.log gpurun_out/r5r_m6_1.log gpurun_out/r5r_base_2.log gpurun_out/r5r_m6_2.log; do echo "$f: $(grep -h 'sgpr:' $f)"; done
