#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 kernel-trace CSV (calls, total / mean us), JSON on stdout.
    python tools/kernel_trace_sum.py <run_kernel_trace.csv> [divisor name=value ...]"""
import csv
import json
import sys
from collections import defaultdict

tot, n = defaultdict(int), defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0][:60]
    tot[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    n[k] += 1
out = {k: {"calls": n[k], "total_us": tot[k] / 1e3, "mean_us": tot[k] / 1e3 / n[k]}
       for k in sorted(tot, key=lambda x: -tot[x])}
out["_all_total_us"] = sum(tot.values()) / 1e3
json.dump(out, sys.stdout, indent=1)
