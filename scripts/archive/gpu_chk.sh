source scripts/gpu_check.sh
export TMPDIR=/tmp
rocm-smi --showclocks --showperflevel > gpurun_out/smi.txt 2>&1 || true
run 120 kchk.log python scripts/knn_only.py --points 1e8 --reps 3
run 300 b100_g0.log python bench.py --points 1e8 --k 100 --steps 3 --warmup 1 --graph 0
run 300 b100_g0_nonuma.log env LSKNN_NUMA_BIND=0 python bench.py --points 1e8 --k 100 --steps 3 --warmup 1 --graph 0
run 300 b100_g1.log python bench.py --points 1e8 --k 100 --steps 3 --warmup 1 --graph 1
run 120 kchk2.log python scripts/knn_only.py --points 1e8 --reps 3
