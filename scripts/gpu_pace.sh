# results copy spread over the next k-NN in chunks (LSKNN_OUT_PACE_MS) vs one burst
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
for c in 600 300 0; do
  LSKNN_OUT_PACE_MS=$c run 400 pace_$c.log python -u bench.py --steps 8 --warmup 2 --verify 64
done
