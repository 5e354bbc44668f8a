#!/bin/bash
# Flags-0 greedy (config 5, 1M pods): mid-window list refresh on / off, two rounds.
set -o pipefail
for r in 1 2; do
  for f in 1 0; do
    echo "== refresh $f: $(YODA_GREEDY_REFRESH=$f YODA_GREEDY_DEBUG=1 timeout -k 10 200 python tools/dbg/topk_window_probe.py 1000000 2>&1 | grep -v amdgpu | tail -3 | tr '\n' ' ')" || exit 1
  done
done
