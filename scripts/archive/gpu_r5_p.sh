#!/bin/bash
# Which engine moves the stream's copies (memory-copy trace), and does forcing the result
# copy off the shader engines change the steady state? (SetStream probe, 1B)
source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$PWD/gpurun_out/r5p_trace
mkdir -p $O
run 400 r5p_trace.log timeout -s KILL 360 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O -o run --output-format csv -- python3 -u scripts/stream_d2h_probe.py 1e9 5 copy
ls $O/*/ 2>/dev/null | head; find $O -name "*memory_copy*" | head -3
f=$(find $O -name "*memory_copy_stats.csv" | head -1); [ -n "$f" ] && cat $f | cut -c1-200
f=$(find $O -name "*memory_copy_trace.csv" | head -1); [ -n "$f" ] && head -5 $f | cut -c1-300 && wc -l $f
grep -v amdgpu.ids gpurun_out/r5p_trace.log | grep "copy run"
