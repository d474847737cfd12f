#!/bin/bash
# Checkpoint after overlap + native comm: full GPU suite, smoke, 1B bench, 8-rank gloo
# rehearsal at 2e8 (multi-process flow with the overlapped halo), kernel stats.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 700 f2_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 120 f2_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 400 f2_bench.log python bench.py --steps 10 --warmup 2
run 600 f2_gloo8.log env LSKNN_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --points 2e8 --steps 2 --warmup 1
