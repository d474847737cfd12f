#!/bin/bash
# MFMA vs VALU screening A/B + its test, then PMC of both forms.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 mfma_test.log python -u -m pytest tests/test_gpu_kernels.py -k mfma -v -x --timeout 200 --timeout-method thread
run 300 mfma_ab.log python scripts/mfma_screen_ab.py --points 1e8 --steps 64
run 200 mfma_stats.log timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/mfma_prof -o run --output-format csv -- python3 scripts/mfma_screen_ab.py --points 2e7 --steps 64 --scale 2.8
run 200 mfma_pmc.log timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $PWD/gpurun_out/mfma_pmc -o run --output-format csv -- python3 scripts/mfma_screen_ab.py --points 2e7 --steps 64 --scale 2.8
