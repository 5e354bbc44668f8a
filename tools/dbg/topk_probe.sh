#!/bin/bash
# Window top-k K2 cost vs list depth and the argmax K2 on the same window sizes (diagnostic).
#   usage (through gpurun): bash tools/dbg/topk_probe.sh <outdir>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1
mkdir -p "$OUT"
timeout -k 10 200 python3 "$ROOT/tools/dbg/window_classes.py" 256 512 1024 > "$OUT/argmax_windows.jsonl" 2> "$OUT/argmax.err"
cd /tmp && export TMPDIR=/tmp
for kt in 8 16; do
  YODA_GREEDY_WINDOW=512 YODA_GREEDY_TOPK=$kt timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d "$OUT/tk$kt" -o run --output-format csv \
    -- python3 "$ROOT/tools/dbg/topk_window_probe.py" 100000 > "$OUT/tk$kt.log" 2>&1
done
cd "$ROOT"
for kt in 8 16; do
  echo "== TOPK $kt"; tail -1 "$OUT/tk$kt.log"
  f=$(find "$OUT/tk$kt" -name "*kernel_stats.csv" | head -1)
  head -12 "$f" | cut -d, -f1-5
done
