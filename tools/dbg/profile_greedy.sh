#!/bin/bash
# Kernel-trace summary of the greedy bench (config 5, one GPU).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_greedy
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --workload greedy --no-cpu-baseline > "$OUT/bench.log" 2>&1
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -20 "$OUT/kernel_stats.csv"
tail -1 "$OUT/bench.log"
