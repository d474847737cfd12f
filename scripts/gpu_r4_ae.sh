# round 4 ae: set i+1's bounds + curve keys beside set i's k-NN (LSKNN_PRE_KEYS) — tests, 1B A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 300 ae_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream.py tests/test_gpu_graph.py -m gpu
LSKNN_PRE_KEYS=1 run 420 ae_pk_1.log python -u bench.py --gpus 1 --steps 20 --warmup 5
run 420 ae_base_1.log python -u bench.py --gpus 1 --steps 20 --warmup 5
