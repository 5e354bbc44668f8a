#!/bin/bash
# Where K1's HBM writes go: WRITE_SIZE (and FETCH_SIZE) of the config-3 bench per libyoda build,
# e.g. the release library against write-ablation builds (-DYODA_ABL_K1_NOPART / _NOBS /
# _NOBM: timing/counter builds that skip one kind of store; their picks are wrong).
#   usage: tools/dbg/k1_write_probe.sh "libA.so libB.so ..."
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$ROOT/gpurun_out/k1_write_probe
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for l in $1; do
  b=$(basename "$l" .so)
  for c in WRITE_SIZE FETCH_SIZE; do
    rm -rf "$OUT/$b-$c"
    YODA_LIB_PATH=$(realpath "$ROOT/$l") timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c \
      -d "$OUT/$b-$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline \
      --no-extras --steps 4 --warmup 1 > "$OUT/$b-$c.log" 2>&1 || { tail -5 "$OUT/$b-$c.log"; exit 1; }
    python3 - "$OUT/$b-$c" "$b" "$c" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
for k in ("k1_block_n32", "k_reduce1", "k2_block_n32", "k_reduce2"):
    v = [x for n, xs in acc.items() if n.startswith(k) or ("::" + k) in n for x in xs]
    if v:
        print(f"{sys.argv[2]:24s} {sys.argv[3]:10s} {k:14s} {sum(v) / len(v) * 1024 / 1e6:8.1f} MB/launch")
PY
  done
done
