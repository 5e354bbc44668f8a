#!/bin/bash
# Interleaved A/B of libyoda builds on config-5 greedy (capacity, then flags 0), one process
# per run:  tools/dbg/greedy_ab.sh "a.so b.so" [rounds]
set -o pipefail
LIBS=$1; R=${2:-2}
mkdir -p gpurun_out
for r in $(seq $R); do
  for l in $LIBS; do
    b=$(basename $l .so)
    echo "== $b cap: $(YODA_LIB_PATH=$(realpath $l) timeout -k 10 200 python tools/dbg/greedy_capacity_dbg.py 1000000 2>&1 | tail -1)" || exit 1
    echo "== $b f0: $(YODA_LIB_PATH=$(realpath $l) timeout -k 10 200 python tools/dbg/topk_window_probe.py 1000000 2>&1 | tail -1)" || exit 1
  done
done
