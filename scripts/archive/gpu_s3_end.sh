#!/bin/bash
# Session-3 end checkpoint: full GPU suite, smoke, and the driver's exact bench command.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 900 s3z_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 120 s3z_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
start=$(date +%s.%N)
run 600 s3z_bench.log python3 bench.py --gpus 1 --steps 20 --warmup 5
end=$(date +%s.%N)
echo "driver-command wall: $(python3 -c "print(round($end - $start, 1))") s" | tee -a gpurun_out/summary.log
