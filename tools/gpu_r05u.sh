#!/bin/bash
# Capacity greedy: chunk list depth (8 / 16) x merged depth A/B.
set -o pipefail
O=gpurun_out/${TAG:-r05u}; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for spec in "16 64" "8 64" "8 128" "8 32"; do
    set -- $spec
    echo "tk$1 d$2 $(YODA_GREEDY_DEBUG=1 YODA_LIB_PATH=$(realpath abl/cur.so) YODA_GREEDY_CAP_TOPK=$1 YODA_GREEDY_CAP_DEPTH=$2 timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 2>&1 | grep -E '^flags|restarts' | tail -2 | cut -c1-330 | tr '\n' ' ')" | tee -a $O/tk_ab.txt
  done
done
