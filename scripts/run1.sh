#!/bin/bash
source scripts/gpu_check.sh
run 120 build.log python mpi_cuda_largescaleknn_amd/_build.py
run 900 t1.log python -m pytest tests/test_gpu_kernels.py -x -q -m gpu
run 300 b1.log python bench.py --points 1e8 --steps 2 --warmup 1 --phases --stats
run 400 b2.log python bench.py --steps 2 --warmup 1 --phases --stats
