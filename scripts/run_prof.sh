#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 600 tgpu.log python -m pytest tests/ -q -m gpu -x
run 600 lb8.log python scripts/loopback_phases.py 1e8 8
