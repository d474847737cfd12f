# round 4 l: redistribution after the k-NN (explicit), forced 1-rank RCCL, distributed tests,
# 2-rank gloo rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 600 t_l.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stream.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_forced_dist.py
LSKNN_DIST_BACKEND=nccl run 300 fd_l.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
run 400 g2_l.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --points 2e8 --steps 2 --warmup 1
run 300 s_1e8_l.log python -u bench.py --points 1e8 --steps 20 --warmup 3
