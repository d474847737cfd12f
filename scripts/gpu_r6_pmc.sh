#!/bin/bash
# PMC passes of the grid k-NN kernel at ${PTS:-1e7} uniform points, k = 100, for each
# library in $V ("prod" = the in-tree library, else lib/exp/liblsknn_hip_<name>.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$PWD/gpurun_out/pmc6${TAG}
mkdir -p $O
for v in ${V:-prod base}; do
  if [ "$v" = prod ]; then L=""; else L=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so; fi
  export LSKNN_HIP_LIB=$L
  [ -z "$L" ] && unset LSKNN_HIP_LIB
  timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a_$v -o run --output-format csv -- python3 scripts/knn_ab.py --points ${PTS:-1e7} --k 100 --reps 1 > $O/a_$v.log 2>&1 || exit 1
  timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_WAVE_CYCLES -d $O/b_$v -o run --output-format csv -- python3 scripts/knn_ab.py --points ${PTS:-1e7} --k 100 --reps 1 > $O/b_$v.log 2>&1 || exit 1
done
for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== ${f#$PWD/}"; python3 scripts/pmc_summary.py $f knn_grid; done > $O/summary.txt 2>&1
cat $O/summary.txt
