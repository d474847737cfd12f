"""Per-set timeline of the k-NN kernels in a rocprofv3 kernel trace (gaps, durations).

    python scripts/timeline.py <dir with *kernel_trace.csv> [kernel substring]"""
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "knn_grid"
rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
big = [(s, e, n) for s, e, n in ks if pat in n and (e - s) > 50e6]
print(f"{len(big)} {pat} launches > 50 ms")
prev_end = None
for s, e, n in big:
    between = [(a, b, m) for a, b, m in ks if prev_end is not None and a >= prev_end and b <= s]
    busy = sum(b - a for a, b, _ in between)
    gap = (s - prev_end) / 1e6 if prev_end is not None else 0.0
    print(f"  kernel {(e - s) / 1e6:9.2f} ms   gap before {gap:8.2f} ms   (other kernels in gap {busy / 1e6:7.2f} ms, n={len(between)})")
    prev_end = e
if len(big) > 1:
    print(f"  period {(big[-1][1] - big[0][1]) / 1e6 / (len(big) - 1):.2f} ms per set")
