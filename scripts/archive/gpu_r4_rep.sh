# round 4 rep: repeat the driver's 1B command on a fresh box (run-to-run spread)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 420 rep_1b_1.log python -u bench.py --gpus 1 --steps 20 --warmup 5
run 420 rep_1b_2.log python -u bench.py --gpus 1 --steps 20 --warmup 5
