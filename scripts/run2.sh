#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
run 120 build.log python mpi_cuda_largescaleknn_amd/_build.py
run 300 debug.log python scripts/debug_knn.py
run 900 t2.log python -m pytest tests/test_gpu_kernels.py -q -m gpu
run 300 knn1.log python scripts/knn_only.py --points 1e8 --reps 2
run 300 prof_trace.log rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o trace --output-format csv -- python3 scripts/knn_only.py --points 3e7
run 300 prof_pmc.log rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/prof_pmc -o pmc --output-format csv -- python3 scripts/knn_only.py --points 3e7
