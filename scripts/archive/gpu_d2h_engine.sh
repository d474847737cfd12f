set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/d2h -o run --output-format csv -- python3 scripts/micro/d2h_engine.py > gpurun_out/d2h.log 2>&1 || exit $?
grep "ms$" gpurun_out/d2h.log
python3 - <<'PY'
import csv, glob
kr = list(csv.DictReader(open(glob.glob('gpurun_out/d2h/**/run_kernel_trace.csv', recursive=True)[0])))
mc = list(csv.DictReader(open(glob.glob('gpurun_out/d2h/**/run_memory_copy_trace.csv', recursive=True)[0])))
ev = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'KERNEL ' + r['Kernel_Name'][:30] + ' q' + r['Queue_Id']) for r in kr]
ev += [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'COPY ' + r['Direction']) for r in mc]
ev.sort()
t0 = ev[0][0]
for s, e, nm in ev:
    if e - s > 5e6:
        print(f"{(s - t0) / 1e6:9.1f} {(e - s) / 1e6:8.1f} {nm}")
PY
