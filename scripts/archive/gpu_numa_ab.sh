#!/bin/bash
# NUMA binding of the bench process (utils/numa.py) on / off, 1B k=100, plus the topology seen.
source scripts/gpu_check.sh
export TMPDIR=/tmp
python - > gpurun_out/numa_topo.txt 2>&1 <<'PY'
import os, torch
p = torch.cuda.get_device_properties(0)
print("pci", p.pci_domain_id, p.pci_bus_id, p.pci_device_id, "allowed cpus", len(os.sched_getaffinity(0)), "of", os.cpu_count())
import sys; sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.utils import numa
print("node cpus", numa.device_numa_cpus(0) and (numa.device_numa_cpus(0)[0], len(numa.device_numa_cpus(0)[1])))
print(os.listdir("/sys/devices/system/node") if os.path.isdir("/sys/devices/system/node") else "no node dir")
PY
run 400 numa_on.log python bench.py --steps 3 --warmup 1 --phases
LSKNN_NUMA_BIND=0 run 400 numa_off.log python bench.py --steps 3 --warmup 1 --phases
run 400 numa_on2.log python bench.py --steps 3 --warmup 1 --phases
