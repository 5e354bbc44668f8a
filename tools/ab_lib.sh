#!/bin/bash
# Interleaved A/B of several libyoda builds on the config-3 bench (one process per run).
#   usage: tools/ab_lib.sh "libA.so libB.so ..." [rounds]
set -o pipefail
LIBS=$1; R=${2:-3}
mkdir -p gpurun_out
for r in $(seq $R); do
  for l in $LIBS; do
    b=$(basename $l .so)
    YODA_LIB_PATH=$(realpath $l) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 \
      > gpurun_out/ab_$b.json 2>gpurun_out/ab_$b.err || { tail -5 gpurun_out/ab_$b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$b.json').read().strip().splitlines()[-1]); print('$b', round(d['ms_per_step'],3), 'ms  k1', round(d['roofline']['k1_avg_ms'],3), 'k2', round(d['roofline']['k2_avg_ms'],3))"
  done
done
