#!/bin/bash
# Derived utilisation metrics of the k-NN kernel (1e8 uniform, k=100), one counter pass each.
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
run 120 pmcd1.log timeout -s KILL 110 rocprofv3 --pmc VALUBusy SALUBusy VALUUtilization OccupancyPercent -d $O/pmcd1 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
run 120 pmcd2.log timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmcd2 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
run 120 pmcd3.log timeout -s KILL 110 rocprofv3 --pmc LDSBankConflict SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $O/pmcd3 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
