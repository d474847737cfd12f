"""Overlap of host-to-device copies with kernels in a rocprofv3 trace.

    python scripts/trace_overlap.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv>

Prints, per copy burst, how much of its time runs concurrently with some kernel."""
import csv
import glob
import sys

d = sys.argv[1]
kt = list(csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0])))
mt = list(csv.DictReader(open(glob.glob(f"{d}/*memory_copy_trace.csv")[0])))
kern = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in kt)
copies = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "")))
                for r in mt)


def merged(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


K = merged([(s, e) for s, e, _ in kern])


def overlap(s, e):
    tot = 0
    for ks, ke in K:
        if ke <= s:
            continue
        if ks >= e:
            break
        tot += min(e, ke) - max(s, ks)
    return tot


big = [c for c in copies if c[1] - c[0] > 1_000_000]  # > 1 ms
tot_c = sum(e - s for s, e, _ in big)
tot_o = sum(overlap(s, e) for s, e, _ in big)
print(f"copies > 1 ms: {len(big)}, {tot_c / 1e6:.1f} ms total, {tot_o / 1e6:.1f} ms "
      f"({100.0 * tot_o / max(tot_c, 1):.0f} %) concurrent with kernels")
for s, e, dirn in big[:40]:
    print(f"  {dirn:24s} {(e - s) / 1e6:8.2f} ms  overlapped {overlap(s, e) / 1e6:8.2f} ms")
