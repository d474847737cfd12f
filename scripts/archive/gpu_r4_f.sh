# round 4 f: one rank's whole ref-algo ring share at 1B / 8 (8 rounds of 125M x 125M, k=100)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 200 ref_ring_1e8_8.log python -u scripts/ref_ring_rank.py 1e8 8
run 900 ref_ring_1e9_8.log python -u scripts/ref_ring_rank.py 1e9 8
