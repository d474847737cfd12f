#!/bin/bash
# Loopback 8 ranks x 1.25e8 points with kernel counters (failed lanes, backstop queries).
source scripts/gpu_check.sh
export TMPDIR=/tmp
run 500 lb8_1b_stats.log python scripts/loopback_phases.py 1e9 8 --stats
