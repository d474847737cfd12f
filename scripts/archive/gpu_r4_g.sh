# round 4 g: launch rehearsal of the driver's multi-GPU commands with the round-4 halo /
# stream code: N ranks on ONE GPU over gloo (host-staged), torchrun as the driver runs it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 400 g2_2e8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2 --points 2e8 --steps 2 --warmup 1
run 400 g4_2e8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29552 bench.py --gpus 4 --points 2e8 --steps 2 --warmup 1
run 500 g8_2e8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29553 bench.py --gpus 8 --points 2e8 --steps 2 --warmup 1
run 900 g8_1b.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29554 bench.py --gpus 8 --steps 2 --warmup 1
