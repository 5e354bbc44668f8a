#!/bin/bash
# e2e split (upload / run / picks) for several libyoda builds on one box.
#   usage: tools/dbg/e2e_ab.sh "libA.so libB.so" [rounds]
set -o pipefail
for r in $(seq ${2:-2}); do
  for l in $1; do
    echo -n "$(basename $l .so): "
    YODA_LIB_PATH=$(realpath $l) timeout -k 10 200 python tools/dbg/e2e_split.py 2>/dev/null | tail -1 || exit 1
  done
done
