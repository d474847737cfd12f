#!/bin/bash
# Loopback 8 ranks x 1.25e8 points (1B) on one MI355X: phase times, halo counts and a
# kernel trace (per-rank local k-NN vs re-query kernel time).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 500 lb8_1b.log python scripts/loopback_phases.py 1e9 8
run 500 lb8_1b_trace.log timeout -s KILL 480 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/lb8_1b -o run --output-format csv -- python3 scripts/loopback_phases.py 1e9 8 --nomarks
