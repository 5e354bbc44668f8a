#!/bin/bash
# Interleaved A/B of env knobs on the config-5 capacity greedy (the A/B build libyoda_ab.so
# reads the YODA_* knobs).   usage: tools/ab_greedy.sh "VAR=a VAR2=b" "VAR=c" ... (rounds 2)
set -o pipefail
mkdir -p gpurun_out
LIB=$(realpath kubernetes-scheduler_amd/yoda_amd/libyoda_ab.so)
for r in 1 2; do
  for cfg in "$@"; do
    out=$(env YODA_LIB_PATH=$LIB $cfg timeout -k 10 300 python tools/greedy_prof.py --flags 1 2>&1 | grep "^flags") || { echo "failed: $cfg"; exit 1; }
    echo "$cfg :: $out"
  done
done
