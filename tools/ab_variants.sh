#!/bin/bash
# Interleaved A/B of several libyoda builds on tools/variants.py workloads (same box).
#   usage: tools/ab_variants.sh "libA.so libB.so ..." "variant ..." [rounds]
set -o pipefail
LIBS=$1; VARS=$2; R=${3:-2}
mkdir -p gpurun_out
for r in $(seq $R); do
  for l in $LIBS; do
    b=$(basename $l .so)
    YODA_LIB_PATH=$(realpath $l) timeout -k 10 300 python tools/variants.py $VARS --steps 5 \
      > gpurun_out/abv_$b.jsonl 2>gpurun_out/abv_$b.err || { tail -5 gpurun_out/abv_$b.err; exit 1; }
    python3 -c "
import json
for line in open('gpurun_out/abv_$b.jsonl'):
    d = json.loads(line)
    print('$b', d['variant'], round(d['ms_per_step'], 3), 'ms  k1', round(d['k1_ms'], 3), 'k2', round(d['k2_ms'], 3))"
  done
done
