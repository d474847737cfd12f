#!/bin/bash
# HIP-graph single-rank step: graph test, full GPU suite, smoke, benches graph on/off.
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 300 tests_graph.log python -u -m pytest tests/test_gpu_graph.py -v -x --timeout 120 --timeout-method thread
run 600 tests_gpu.log python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
for cfg in "1e6 8 10 2" "1e7 16 10 2" "1e8 100 3 1"; do set -- $cfg
  for gr in 0 1; do run 300 g_${1}_k${2}_g$gr.log python bench.py --points $1 --k $2 --steps $3 --warmup $4 --graph $gr; done
done
run 600 g_1b.log python bench.py
