set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/mfma_c8.log
: > $O
timeout -k 10 200 python scripts/mfma_check.py --points 1e6 --k 100 --oracle 1000 --reps 2 >> $O 2>&1 &&
timeout -k 10 200 python scripts/mfma_check.py --points 1e8 --k 100 --reps 3 --only mfma >> $O 2>&1
rc=$?
cat $O
exit $rc
