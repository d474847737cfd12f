#!/bin/bash
# PMC counters of the current k-NN kernel (3e7 uniform points, k=100), one set per pass.
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
P="python3 scripts/knn_only.py --points 3e7"
run 90 pmc1.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $O/pmc1 -o run --output-format csv -- $P
run 90 pmc2.log timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/pmc2 -o run --output-format csv -- $P
run 90 pmc3.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SENDMSG -d $O/pmc3 -o run --output-format csv -- $P
for d in pmc1 pmc2 pmc3; do f=$(ls $O/$d/*counter_collection.csv | head -1); python scripts/pmc_summary.py $f knn_rows > $O/${d}_summary.txt; done
cat $O/pmc*_summary.txt
