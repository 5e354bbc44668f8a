#!/bin/bash
# Capacity greedy (config 5, flags 1) on one GPU: per-window host trace, failed certificates,
# kernel totals.
set -o pipefail
O=gpurun_out/r05l; rm -rf $O; mkdir -p $O
export YODA_GREEDY_DEBUG=1
YODA_GREEDY_TRACE=$O/windows.txt timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 > $O/plain.txt 2>&1 || { tail -5 $O/plain.txt; exit 1; }
cat $O/plain.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/greedy_prof.py --flags 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_trace_sum.py $T > $O/kernels.json
python3 - $T > $O/gaps.txt <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(sys.argv[1])))
busy = sum(e - s for s, e in rows)
span = rows[-1][1] - rows[0][0]
print(f"kernels {len(rows)} busy {busy/1e6:.1f} ms span {span/1e6:.1f} ms")
PY
cat $O/gaps.txt; head -c 1500 $O/kernels.json
find $O/prof -name '*kernel_trace.csv' -delete
