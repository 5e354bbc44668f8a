#!/bin/bash
# picks download A/B: direct pageable copies (0) vs pinned staging + pool (1) / one thread (2)
set -o pipefail
O=gpurun_out/r05o; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for v in 0 1 2; do
    echo "dl$v $(YODA_LIB_PATH=$(realpath abl/cur.so) YODA_DL_STAGE=$v timeout -k 10 200 python3 tools/dbg/e2e_split.py 2>&1 | tail -1)" | tee -a $O/e2e_ab.txt
  done
done
