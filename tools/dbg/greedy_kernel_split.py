"""Per-kernel split of a greedy kernel trace (rocprofv3 run_kernel_trace.csv): calls, mean
duration by grid, total ms.  usage: python greedy_kernel_split.py <trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    key = r["Kernel_Name"].split("(")[0][:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by[key].append((int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), d))
tot = sorted(by.items(), key=lambda kv: -sum(x[2] for x in kv[1]))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
t1 = max(int(r["End_Timestamp"]) for r in rows)
print(f"trace span {(t1 - t0) / 1e6:.1f} ms, kernels {sum(len(v) for v in by.values())}")
for k, L in tot[:14]:
    hist = collections.defaultdict(list)
    for gx, gy, d in L:
        hist[(gx, gy)].append(d)
    top = sorted(hist.items(), key=lambda kv: -len(kv[1]))[:3]
    desc = ", ".join(f"{g}: n={len(v)} {sum(v) / len(v):.1f}us" for g, v in top)
    print(f"{sum(x[2] for x in L) / 1e3:9.1f} ms {len(L):6d}  {k}  [{desc}]")
