# PMC passes of the k-NN kernels at 1e7 uniform points, k = 100 (one kernel per run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$PWD/gpurun_out/pmc5${TAG}
mkdir -p $O
for kern in ${KERNS:-mfma sgpr}; do
timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a_$kern -o run --output-format csv -- python3 scripts/knn_ab.py --points ${PTS:-1e7} --k 100 --reps 1 > $O/a_$kern.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES -d $O/b_$kern -o run --output-format csv -- python3 scripts/knn_ab.py --points ${PTS:-1e7} --k 100 --reps 1 > $O/b_$kern.log 2>&1 || exit 1
done
for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== ${f#$PWD/}"; python3 scripts/pmc_summary.py $f knn_; done > $O/summary.txt 2>&1
cat $O/summary.txt
