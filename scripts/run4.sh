#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
run 120 build.log python mpi_cuda_largescaleknn_amd/_build.py
run 900 t4.log python -m pytest tests/test_gpu_distributed.py -q -m gpu -x
run 600 b4.log python bench.py --steps 2 --warmup 1 --phases --stats
