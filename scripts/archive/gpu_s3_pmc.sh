#!/bin/bash
# PMC of the final session-3 k-NN kernel (2-wave blocks), 3e7 uniform points, k=100.
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
run 120 s3pmc1.log timeout -s KILL 110 rocprofv3 --pmc VALUBusy SALUBusy VALUUtilization OccupancyPercent -d $O/s3pmc1 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
run 120 s3pmc2.log timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/s3pmc2 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
