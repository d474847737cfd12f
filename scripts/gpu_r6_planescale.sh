#!/bin/bash
# Rotated plane frame at larger n (denser planes: the k-NN radius shrinks toward the box
# margin rotate_margin): 2e8 and 5e8 tilted plane, k = 100 and 48, frame on / off.
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1 LSK_DISTS=tilted_plane LSK_REPS=3
for n in 2e8 5e8; do for f in 1 0; do
  run 300 r6ps_${n}_$f.log env LSKNN_FLAT_FRAME=$f python -u scripts/dist_robustness.py $n 100 48 || exit $?
done; done
for f in gpurun_out/r6ps_*.log; do echo "== $(basename $f)"; grep -h "^{'dist'" $f; done
