#!/bin/bash
# Round-3 knob A/B: flags-0 refresh period / bar, capacity list depth.
set -o pipefail
for r in 1 2; do
  for cfg in "16 32" "8 16" "4 16" "8 8"; do
    set -- $cfg
    echo "== f0 every $1 min $2: $(YODA_GREEDY_REFRESH_EVERY=$1 YODA_GREEDY_REFRESH_MIN=$2 timeout -k 10 200 python tools/dbg/topk_window_probe.py 1000000 2>&1 | tail -1)" || exit 1
  done
  for kt in 16 8; do
    echo "== cap topk $kt: $(YODA_GREEDY_CAP_TOPK=$kt timeout -k 10 200 python tools/dbg/greedy_capacity_dbg.py 1000000 2>&1 | tail -1)" || exit 1
  done
done
