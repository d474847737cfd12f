"""How much of the halo exchange runs under the local k-NN, from a rocprofv3 kernel trace.

    python scripts/halo_overlap_trace.py <dir with *_kernel_trace.csv>

For every halo-side kernel (a-priori radius bounds, publish levels, halo filter, counts,
pack) prints the share of its execution time that overlaps some knn_rows_kernel
execution, and the same for the whole side-stream span per k-NN launch."""
import csv
import glob
import sys

rows = list(csv.DictReader(open(glob.glob(f"{sys.argv[1]}/*kernel_trace.csv")[0])))
SIDE = ("leaf_radius_ub", "halo_mask", "mask_counts", "halo_pack")
knn = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
             if "knn_rows_kernel" in r["Kernel_Name"])
side = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:])
              for r in rows if any(s in r["Kernel_Name"] for s in SIDE))


def covered(s, e):
    c = 0
    for ks, ke in knn:
        lo, hi = max(s, ks), min(e, ke)
        if hi > lo:
            c += hi - lo
    return c


tot = sum(e - s for s, e, _ in side)
cov = sum(min(covered(s, e), e - s) for s, e, _ in side)
by = {}
for s, e, n in side:
    a = by.setdefault(n, [0, 0, 0])
    a[0] += 1
    a[1] += e - s
    a[2] += min(covered(s, e), e - s)
for n, (c, t, v) in sorted(by.items()):
    print(f"{n:42s} launches {c:3d}  {t / 1e6:8.3f} ms  under k-NN {100.0 * v / max(t, 1):5.1f} %")
print(f"halo-side kernels: {tot / 1e6:.3f} ms total, {100.0 * cov / max(tot, 1):.1f} % under knn_rows_kernel "
      f"({len(knn)} k-NN launches, {sum(e - s for s, e in knn) / 1e6:.1f} ms)")
