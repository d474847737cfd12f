#!/bin/bash
# Measures the BASELINE.md table on one MI355X (writes gpurun_out/table_*.json lines).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 120 build.log python mpi_cuda_largescaleknn_amd/_build.py
run 300 table_10m_k16.log python bench.py --points 1e7 --k 16 --steps 5 --warmup 1
run 300 table_10m_k16_ring.log python bench.py --points 1e7 --k 16 --steps 2 --warmup 1 --mode ring
run 300 table_100m.log python bench.py --points 1e8 --steps 3 --warmup 1 --phases
run 300 table_100m_pre.log python bench.py --points 1e8 --steps 3 --warmup 1 --variant prepartitioned
run 900 table_1b.log python bench.py --steps 3 --warmup 1 --phases
run 300 table_1m_k8.log python bench.py --points 1e6 --k 8 --steps 5 --warmup 2
