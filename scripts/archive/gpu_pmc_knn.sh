#!/bin/bash
# PMC counters of the k-NN kernel (3e7 uniform points, k=100), one counter set per pass.
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
run 90 pmc1.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $O/pmc1 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7
run 90 pmc2.log timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/pmc2 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7
for d in pmc1 pmc2; do f=$(ls $O/$d/*counter_collection.csv | head -1); python scripts/pmc_summary.py $f knn_rows > $O/${d}_summary.txt; done
