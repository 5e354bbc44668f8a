#!/bin/bash
# Deep merged lists for the capacity windows: greedy tests, then depth A/B (0 = the chunks' 16).
set -o pipefail
O=gpurun_out/r05p; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "greedy" > $O/pytest_greedy.txt 2>&1 || { tail -30 $O/pytest_greedy.txt; exit 1; }
tail -1 $O/pytest_greedy.txt
for r in 1 2; do
  for d in 0 32 64 128; do
    echo "depth$d $(YODA_GREEDY_DEBUG=1 YODA_LIB_PATH=$(realpath abl/cur.so) YODA_GREEDY_CAP_DEPTH=$d timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 2>&1 | grep -E '^flags|restarts' | tail -2 | cut -c1-200 | tr '\n' ' ')" | tee -a $O/depth_ab.txt
  done
done
