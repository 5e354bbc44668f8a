#!/bin/bash
# Kernel trace of the capacity greedy alone (config 5, 1M pods), then its per-kernel split.
#   usage (through gpurun): bash tools/dbg/profile_greedy_cap.sh <outdir>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o run --output-format csv \
  -- python3 "$ROOT/tools/dbg/greedy_capacity_dbg.py" 1000000 > "$OUT/run.log" 2>&1
cd "$ROOT"
tail -2 "$OUT/run.log"
python3 tools/dbg/greedy_kernel_split.py $(find "$OUT/tr" -name "*kernel_trace.csv") | tee "$OUT/split.txt"
