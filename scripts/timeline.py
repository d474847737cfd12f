"""Per-set timeline of the k-NN kernels in a rocprofv3 kernel trace (gaps, durations).

    python scripts/timeline.py <dir with *kernel_trace.csv or *.db> [kernel substring] [--gaps]

--gaps also lists, for every gap between two consecutive big k-NN kernels, the kernels
that ran in it and the idle time (no kernel running on the device)."""
import csv
import glob
import sqlite3
import sys


def load(d):
    dbs = glob.glob(f"{d}/**/*.db", recursive=True)
    if dbs:
        c = sqlite3.connect(dbs[0])
        return sorted((int(s), int(e), n) for s, e, n in c.execute("select start, end, name from kernels"))
    rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)


def idle_ns(spans, lo, hi):
    """Time in [lo, hi) not covered by any span."""
    t, idle = lo, 0
    for a, b in sorted(spans):
        if b <= t:
            continue
        if a > t:
            idle += min(a, hi) - t
        t = max(t, b)
        if t >= hi:
            break
    return idle + max(0, hi - t)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    d = args[0]
    pat = args[1] if len(args) > 1 else "knn_grid"
    gaps = "--gaps" in sys.argv
    ks = load(d)
    big = [(s, e, n) for s, e, n in ks if pat in n and (e - s) > 20e6]
    print(f"{len(big)} {pat} launches > 20 ms")
    prev_end = None
    for s, e, n in big:
        between = [(a, b, m) for a, b, m in ks if prev_end is not None and a >= prev_end and b <= s]
        busy = sum(b - a for a, b, _ in between)
        gap = (s - prev_end) / 1e6 if prev_end is not None else 0.0
        idle = idle_ns([(a, b) for a, b, _ in between], prev_end, s) / 1e6 if prev_end is not None else 0.0
        print(f"  kernel {(e - s) / 1e6:9.2f} ms   gap before {gap:8.2f} ms   (other kernels {busy / 1e6:7.2f} ms, "
              f"n={len(between)}, device idle {idle:7.2f} ms)")
        if gaps and between:
            agg = {}
            for a, b, m in between:
                k = m.split("(")[0][-60:]
                agg[k] = agg.get(k, 0) + (b - a)
            for k, v in sorted(agg.items(), key=lambda x: -x[1])[:12]:
                print(f"        {v / 1e6:8.3f} ms  {k}")
        prev_end = e
    if len(big) > 1:
        print(f"  period {(big[-1][1] - big[0][1]) / 1e6 / (len(big) - 1):.2f} ms per set")


if __name__ == "__main__":
    main()
