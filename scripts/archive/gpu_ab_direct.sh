#!/bin/bash
# Direct host output (k-NN kernel writes distances over PCIe) vs device buffer + copy:
# k-NN kernel time per point vs k, and the bench at both settings around the crossover.
source scripts/gpu_check.sh
export TMPDIR=/tmp
for k in 8 16 32 48 64 80 100 128; do
run 120 kt_$k.log python scripts/knn_only.py --points 1e8 --k $k --reps 2
done
for k in 48 64 80; do for d in 0 1; do
run 200 ab_100m_k${k}_d$d.log python bench.py --points 1e8 --k $k --steps 3 --warmup 1 --direct-out $d
done; done
