"""Per-rank GPU kernel time of a loopback kernel trace (scripts/gpu_lb_scaling.sh):
the second repetition's kernels between the last 1-rank-sized k-NN launches, divided by P."""
import collections
import csv
import sys

path, P = sys.argv[1], int(sys.argv[2])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
knn = [i for i, r in enumerate(rows) if "knn_rows_kernel<32, 1>" in r["Kernel_Name"]]
# launches: rep1 P local passes, rep2 P local passes, then the 1-rank reference pass
rep2_first = knn[P]
rep1_last_req = max(i for i, r in enumerate(rows[:rep2_first]) if "knn_rows_kernel<32, 2>" in r["Kernel_Name"])
end = max(i for i, r in enumerate(rows[:knn[-1]]) if "knn_rows_kernel<32, 2>" in r["Kernel_Name"])
win = rows[rep1_last_req + 1:end + 1]
agg = collections.defaultdict(float)
for r in win:
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    agg[nm.split("(")[0][:48]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(agg.values())
single = (int(rows[knn[-1]]["End_Timestamp"]) - int(rows[knn[-1]]["Start_Timestamp"])) / 1e6
print(f"P={P}: kernel time per rank {tot / P:.1f} ms (k-NN local {agg.get('knn_rows_kernel<32, 1>', 0) / P:.1f}, "
      f"re-query {agg.get('knn_rows_kernel<32, 2>', 0) / P:.1f}); 1-rank k-NN pass {single:.1f} ms -> ideal {single / P:.1f}")
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:12]:
    print(f"   {v / P:8.2f} ms/rank  {k}")
