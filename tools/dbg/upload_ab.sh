#!/bin/bash
# Flags-0 greedy (config 5): upload packing threads per window (YODA_UPLOAD_MIN_RANGE).
set -o pipefail
for r in 1 2; do
  for m in 4096 1024 512; do
    echo "== min_range $m: $(YODA_UPLOAD_MIN_RANGE=$m YODA_GREEDY_DEBUG=1 timeout -k 10 200 python tools/dbg/topk_window_probe.py 1000000 2>&1 | grep -v amdgpu | grep -v refreshes | tail -2 | tr '\n' ' ')" || exit 1
  done
done
