#!/bin/bash
# Session 3: the BASELINE.md table with the final build (unordered: stream of sets default).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 s3t_1m_k8.log python bench.py --points 1e6 --k 8 --steps 20 --warmup 5
run 300 s3t_10m_k16.log python bench.py --points 1e7 --k 16 --steps 20 --warmup 5
run 300 s3t_100m_k100.log python bench.py --points 1e8 --steps 20 --warmup 5
run 300 s3t_100m_pre.log python bench.py --points 1e8 --steps 20 --warmup 5 --variant prepartitioned
