#!/bin/bash
# Restart-window sizing A/B on the config-5 capacity greedy (YODA_GREEDY_GROW_PCT values).
set -o pipefail
for r in 1 2; do
  for g in ${GROWS:-0 100 130 160}; do
    echo "== grow $g: $(YODA_GREEDY_GROW_PCT=$g timeout -k 10 200 python tools/dbg/greedy_capacity_dbg.py 1000000 2>&1 | tail -1)" || exit 1
  done
done
