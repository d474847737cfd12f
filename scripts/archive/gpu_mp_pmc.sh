#!/bin/bash
# Multi-process GPU tests (gloo staging, ranks sharing cuda:0) + PMC / kernel-trace
# evidence of the current k-NN kernel (3e7 / 1e8 uniform points, k=100).
source scripts/gpu_check.sh
export TMPDIR=/tmp
O=$PWD/gpurun_out
run 400 tests_mp.log python -u -m pytest tests/test_gpu_multiprocess.py -v -x --timeout 300 --timeout-method thread
run 90 pmc1.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $O/pmc1 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7
run 90 pmc2.log timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/pmc2 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7
run 90 pmc3.log timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM GRBM_COUNT -d $O/pmc3 -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7
for d in pmc1 pmc2 pmc3; do f=$(ls $O/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && python scripts/pmc_summary.py $f knn_rows > $O/${d}_summary.txt; done
run 300 prof_stats.log rocprofv3 --kernel-trace --stats -d $O/prof_stats -o run --output-format csv -- python3 bench.py --points 1e8 --steps 2 --warmup 1
