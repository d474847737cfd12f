#!/bin/bash
# BASELINE table rows with the final round-2 build (single MI355X, bench.py defaults).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 200 tb_1m_k8.log python bench.py --points 1e6 --k 8 --steps 20 --warmup 3
run 200 tb_10m_k16.log python bench.py --points 1e7 --k 16 --steps 20 --warmup 3
run 300 tb_100m_k100.log python bench.py --points 1e8 --k 100 --steps 10 --warmup 2
run 300 tb_100m_pre.log python bench.py --points 1e8 --k 100 --steps 10 --warmup 2 --variant prepartitioned
