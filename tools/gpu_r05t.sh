#!/bin/bash
# Capacity greedy at depth 64: greedy tests, the lost-node witness filter, window growth A/B.
set -o pipefail
O=gpurun_out/${TAG:-r05t}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "greedy" > $O/pytest_greedy.txt 2>&1 || { tail -30 $O/pytest_greedy.txt; exit 1; }
tail -1 $O/pytest_greedy.txt
for r in 1 2; do
  for g in 130 115 150; do
    echo "grow$g $(YODA_GREEDY_DEBUG=1 YODA_LIB_PATH=$(realpath abl/cur.so) YODA_GREEDY_GROW_PCT=$g timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 2>&1 | grep -E '^flags|restarts' | tail -2 | cut -c1-330 | tr '\n' ' ')" | tee -a $O/grow_ab.txt
  done
done
