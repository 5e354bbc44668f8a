#!/bin/bash
# Capacity greedy defaults (chunk lists 8, merged 64, borrowed lists): greedy tests + timing.
set -o pipefail
O=gpurun_out/${TAG:-r05v}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "greedy" > $O/pytest_greedy.txt 2>&1 || { tail -30 $O/pytest_greedy.txt; exit 1; }
tail -1 $O/pytest_greedy.txt
for r in 1 2 3; do
  echo "cur $(YODA_GREEDY_DEBUG=1 timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 0 2>&1 | grep -E '^flags|restarts' | cut -c1-200 | tr '\n' ' ')" | tee -a $O/timing.txt
done
