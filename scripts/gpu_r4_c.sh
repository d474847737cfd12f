# round 4 c: debug the device gate under capture and the boundary-first halo on loopback
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 300 debug_r4.log python -u scripts/debug_r4.py
