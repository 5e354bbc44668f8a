#!/bin/bash
# e2e A/B on one box: the committed upload (head) vs the working tree (cur).
set -o pipefail
O=gpurun_out/r05e2e; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for lab in head cur; do
    lib=abl/at_head.so; [ $lab = cur ] && lib=kubernetes-scheduler_amd/yoda_amd/libyoda.so
    echo "$lab $(YODA_UPLOAD_DEBUG=1 YODA_LIB_PATH=$(realpath $lib) timeout -k 10 200 python3 tools/dbg/e2e_split.py 2>&1 | tail -2 | tr '\n' ' ')" | tee -a $O/e2e_ab.txt
  done
done
