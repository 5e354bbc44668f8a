#!/bin/bash
# e2e A/B on one box: pool workers spinning 2 ms before parking vs parking at once.
set -o pipefail
O=gpurun_out/r05spin; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for v in 2000 0; do
    echo "spin$v $(YODA_POOL_SPIN_US=$v YODA_UPLOAD_DEBUG=1 YODA_LIB_PATH=$(realpath abl/cur.so) timeout -k 10 200 python3 tools/dbg/e2e_split.py 2>&1 | tail -2 | tr '\n' ' ')" | tee -a $O/e2e_ab.txt
  done
done
