# round 4 s: the previous set's result copy beside the k-NN instead of the build (1B, 1e8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
for r in 1 2; do
  LSKNN_OUT_AFTER_BUILD=0 run 400 oab0_1b_$r.log python -u bench.py --steps 10 --warmup 3
  LSKNN_OUT_AFTER_BUILD=1 run 400 oab1_1b_$r.log python -u bench.py --steps 10 --warmup 3
done
LSKNN_OUT_AFTER_BUILD=0 run 300 oab0_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 3
LSKNN_OUT_AFTER_BUILD=1 run 300 oab1_1e8.log python -u bench.py --points 1e8 --steps 20 --warmup 3
