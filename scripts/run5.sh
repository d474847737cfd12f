#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 120 build.log python mpi_cuda_largescaleknn_amd/_build.py
run 900 t5.log python -m pytest tests/ -q -m gpu
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 b_cfg2_ours.log python bench.py --points 1e7 --k 16 --steps 5 --warmup 1
run 300 b_cfg2_ref.log python bench.py --points 1e7 --k 16 --steps 2 --warmup 1 --mode ring
run 300 b_100m_ours.log python bench.py --points 1e8 --steps 3 --warmup 1
run 900 b_100m_ref.log python bench.py --points 1e8 --steps 1 --warmup 0 --mode ring --phases
