#!/bin/bash
# e2e split with the deferred pod copy on the side stream (default) vs after the kernels,
# then a copy/kernel timeline of the default.
set -o pipefail
O=gpurun_out/r05m; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for spec in "side|" "noside|YODA_SIDE_COPY=0"; do
    IFS='|' read -r lab envs <<< "$spec"
    env YODA_LIB_PATH=$(realpath abl/cur.so) $envs timeout -k 10 200 python3 tools/dbg/e2e_split.py > $O/e2e_$lab.txt 2>&1 || { cat $O/e2e_$lab.txt; exit 1; }
    echo "$lab $(tail -1 $O/e2e_$lab.txt)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/$O/tl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/dbg/e2e_split.py > $GRAFT_REPO_ROOT/$O/tl.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/tl.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - $O/tl > $O/timeline.txt <<'PY'
import csv, glob, sys
d = sys.argv[1]
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40]))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "") + " " + r.get("Size", "")))
ev.sort()
# the last 60 events = the last e2e iteration or so
last = ev[-60:]
t0 = last[0][0]
for s, e, n in last:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {n}")
PY
cat $O/timeline.txt
find $O/tl -name '*.csv' -delete
