#!/bin/bash
# Capacity greedy: exact fallback instead of a restart when few of the next window pods are
# uncertified already (YODA_GREEDY_CAP_SCAN / _MAX), against restart-only.
set -o pipefail
for r in 1 2; do
  for cfg in "0 1" "32 1" "64 3" "16 0"; do
    set -- $cfg
    echo "== scan $1 max $2: $(YODA_GREEDY_CAP_SCAN=$1 YODA_GREEDY_CAP_SCAN_MAX=$2 timeout -k 10 200 python tools/dbg/greedy_capacity_dbg.py 1000000 2>&1 | tail -1)" || exit 1
  done
done
