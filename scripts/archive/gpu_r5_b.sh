# kernel-trace of knn_mfma experiment variants at 1e7 (wrong results by design: timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$PWD/gpurun_out/mfx
mkdir -p $O
for v in base x1 x2 x3; do
  if [ $v = base ]; then L=""; else L=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 scripts/mfma_check.py --points 1e7 --k 100 --reps 2 --only mfma > $O/$v.log 2>&1 || exit 1
  echo "== $v" >> $O/summary.txt
  grep -h "knn_mfma\|knn_exact" $(find $O/$v -name "*kernel_stats.csv") | cut -d, -f1-4 >> $O/summary.txt
done
cat $O/summary.txt
