#!/bin/bash
# Session 3: is the k-NN kernel's occupancy (60.6 % of 32 waves/CU measured, 87.5 % cap)
# limited by the runtime's scratch allocation? knn_only 1e8 with the default scratch
# limit vs a raised one, plus one OccupancyPercent pass each.
source scripts/gpu_check.sh
export TMPDIR=/tmp
for round in 1 2; do
  run 150 s3occ_def_$round.log python scripts/knn_only.py --points 1e8 --reps 3
  run 150 s3occ_big_$round.log env HSA_SCRATCH_SINGLE_LIMIT=4294967296 python scripts/knn_only.py --points 1e8 --reps 3
done
run 120 s3occ_pmc_def.log timeout -s KILL 110 rocprofv3 --pmc OccupancyPercent -d $PWD/gpurun_out/s3occ_pmc_def -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
run 120 s3occ_pmc_big.log env HSA_SCRATCH_SINGLE_LIMIT=4294967296 timeout -s KILL 110 rocprofv3 --pmc OccupancyPercent -d $PWD/gpurun_out/s3occ_pmc_big -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1
