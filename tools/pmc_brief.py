#!/usr/bin/env python3
"""One line per kernel of a pmc_summary.json: time, HBM bytes, issue utilisation."""
import json
import sys

d = json.load(open(sys.argv[1]))
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("avg_ns", 0) * kv[1].get("calls", 0)):
    if "avg_ns" not in v:
        continue
    print(f"{k[:40]:40s} {v['avg_ns'] / 1e3:8.1f} us x{v['calls']:<4d} "
          f"rd {v.get('hbm_read_bytes_corrected_x2', 0) / 1e6:7.1f} MB "
          f"wr {v.get('hbm_write_bytes', 0) / 1e6:7.1f} MB "
          f"valu {v.get('valu_issue_util', 0):.2f} salu {v.get('salu_issue_util', 0):.2f}")
