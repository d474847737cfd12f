# PMC: grid kernel vs rows kernel on 3e7 uniform points, k=100 (one pass each).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$PWD/gpurun_out/r3pmc
mkdir -p $O
for g in 1 0; do
timeout -s KILL 110 rocprofv3 --pmc VALUBusy SALUBusy VALUUtilization OccupancyPercent -d $O/a$g -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid $g > $O/a$g.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/b$g -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid $g > $O/b$g.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d $O/c$g -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid $g > $O/c$g.log 2>&1 || echo "pass c failed (counter names?)"
done
for f in $(find $O -name "*counter_collection.csv"); do echo "== $f"; python3 scripts/pmc_summary.py $f knn_; done > $O/summary.txt 2>&1
cat $O/summary.txt
