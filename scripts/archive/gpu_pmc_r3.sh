# PMC of the 3-level grid kernel vs the rows kernel, 3e7 uniform points, k=100 (one counter set per pass).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$PWD/gpurun_out/r3pmc2
mkdir -p $O
for g in 1 0; do
timeout -s KILL 110 rocprofv3 --pmc VALUBusy SALUBusy VALUUtilization OccupancyPercent -d $O/a$g -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid $g > $O/a$g.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $O/b$g -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid $g > $O/b$g.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $O/c$g -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid $g > $O/c$g.log 2>&1 || exit 1
done
for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== ${f#$PWD/}"; python3 scripts/pmc_summary.py $f knn_; done > $O/summary.txt 2>&1
cat $O/summary.txt
