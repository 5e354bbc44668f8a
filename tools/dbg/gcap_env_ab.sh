#!/bin/bash
# Capacity greedy (config 5, 1M pods) under several environment settings, one box.
#   usage: tools/dbg/gcap_env_ab.sh "VAR=a VAR=b ..."   (each word: one run's env assignment)
set -o pipefail
for e in $1; do
  echo -n "$e: "
  env $e timeout -k 10 200 python tools/dbg/greedy_capacity_dbg.py 1000000 2>/dev/null | tail -1 || exit 1
done
