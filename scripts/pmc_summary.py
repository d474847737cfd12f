"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (sum over dispatches)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for name, c in agg.items():
    if pat and pat not in name:
        continue
    print(name)
    for k, v in sorted(c.items()):
        print(f"   {k:28s} {v:.4g}")
    if "SQ_WAVES" in c and c["SQ_WAVES"]:
        w = c["SQ_WAVES"]
        print("   per-wave:", {k: round(v / w) for k, v in c.items() if k.startswith("SQ_INSTS")})
