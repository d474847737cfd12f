# PMC passes of the final grid kernel (row-union culling) at 3e7, kernel trace of the 1B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$PWD/gpurun_out/pmcf
mkdir -p $O
timeout -s KILL 110 rocprofv3 --pmc VALUBusy SALUBusy VALUUtilization OccupancyPercent -d $O/a -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/a.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/b.log 2>&1 || exit 1
for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== ${f#$PWD/}"; python3 scripts/pmc_summary.py $f knn_; done > $O/summary.txt 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --verify 0 > gpurun_out/prof_final_bench.log 2>&1 || exit $?
python3 scripts/timeline.py gpurun_out/prof_final knn_grid > gpurun_out/prof_final_timeline.txt 2>&1
cat $O/summary.txt | head -30
