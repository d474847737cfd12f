# 8 ranks on ONE GPU over gloo (host-staged collectives): rehearsal of the driver's 8-GPU
# launch with the session-2 kernels (torchrun as the driver runs it, and bench.py's own
# self-launch); not an xGMI/RCCL measurement
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 600 g8_2e8_torchrun.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --points 2e8 --steps 2 --warmup 1
run 600 g8_2e8_self.log env LSKNN_DIST_BACKEND=gloo python bench.py --gpus 8 --points 2e8 --steps 2 --warmup 1
run 900 g8_1b_torchrun.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 8 --steps 2 --warmup 1
