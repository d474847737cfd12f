set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/full_tests.log 2>&1; rc=$?; tail -4 gpurun_out/full_tests.log; [ $rc -eq 0 ] || exit $rc
for b in nccl rccl; do LSKNN_DIST_BACKEND=$b timeout -k 10 400 python -u bench.py --force-dist --points 1e8 --steps 6 --warmup 2 > gpurun_out/full_fd_$b.log 2>&1; echo "forced $b"; tail -1 gpurun_out/full_fd_$b.log | cut -c1-700; done
timeout -k 10 300 python -u bench.py --points 1e8 --steps 6 --warmup 2 > gpurun_out/full_1e8.log 2>&1; tail -1 gpurun_out/full_1e8.log | cut -c1-400
O=$PWD/gpurun_out/fullpmc; mkdir -p $O
timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES -d $O/a -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/a.log 2>&1 || echo "pmc a failed"
timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 0 > $O/b.log 2>&1 || echo "pmc b failed"
timeout -s KILL 100 rocprofv3 --pmc VALUBusy SALUBusy VALUUtilization OccupancyPercent -d $O/c -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/c.log 2>&1 || echo "pmc c failed"
timeout -s KILL 100 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES -d $O/d -o run --output-format csv -- python3 scripts/knn_only.py --points 3e7 --reps 1 --grid 1 > $O/d.log 2>&1 || echo "pmc d failed"
for f in $(find $O -name "*counter_collection.csv"); do echo "== $f"; python3 scripts/pmc_summary.py $f knn_; done > $O/summary.txt 2>&1
cat $O/summary.txt | grep -v "^   [A-Z]" | head -60
