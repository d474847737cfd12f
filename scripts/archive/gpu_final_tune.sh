# end-of-session check: full GPU suite, smoke, the driver's 1B bench, the table configs,
# and a kernel-stats profile of the 1B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 900 fin_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu
grep -q " passed" gpurun_out/fin_tests.log && ! grep -q "failed" gpurun_out/fin_tests.log || exit 1
run 200 fin_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run 500 fin_bench_1b.log python -u bench.py --gpus 1 --steps 20 --warmup 5
run 300 fin_bench_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 3
run 200 fin_bench_1e7_k16.log python -u bench.py --points 1e7 --k 16 --steps 20 --warmup 3
run 200 fin_bench_1e6_k8.log python -u bench.py --points 1e6 --k 8 --steps 50 --warmup 5
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --verify 0 > gpurun_out/fin_prof.log 2>&1 || exit $?
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
for v in base tb8 tb12 ec07 ec09; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 300 tune_knn_$v.log python -u scripts/knn_only.py --points 1e8 --reps 4 --grid 1
done
O=$PWD/gpurun_out/s2pmc
mkdir -p $O
timeout -s KILL 110 rocprofv3 --pmc VALUBusy SALUBusy VALUUtilization OccupancyPercent -d $O/a -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/a.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/b.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $O/c -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/c.log 2>&1 || exit 1
for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== ${f#$PWD/}"; python3 scripts/pmc_summary.py $f knn_; done > $O/summary.txt 2>&1
cat $O/summary.txt
