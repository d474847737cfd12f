#!/bin/bash
# Scalar-unit throughput micro + PMC passes of knn_mfma / knn_grid (sgpr) at 1e7, k=100.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5e
mkdir -p $O
timeout -k 10 120 ./scripts/micro/salu > $O/salu.log 2>&1 || exit 1
cat $O/salu.log
for kern in mfma sgpr; do
timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a_$kern -o run --output-format csv -- python3 scripts/mfma_check.py --points 1e7 --k 100 --reps 1 --only $kern > $O/a_$kern.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES SQ_WAVE_CYCLES -d $O/b_$kern -o run --output-format csv -- python3 scripts/mfma_check.py --points 1e7 --k 100 --reps 1 --only $kern > $O/b_$kern.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT32 SQ_WAVES SQ_WAVE_CYCLES -d $O/c_$kern -o run --output-format csv -- python3 scripts/mfma_check.py --points 1e7 --k 100 --reps 1 --only $kern > $O/c_$kern.log 2>&1 || echo "pass c failed for $kern"
done
for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== ${f#$PWD/}"; python3 scripts/pmc_summary.py $f knn_; done > $O/summary.txt 2>&1
cat $O/summary.txt
