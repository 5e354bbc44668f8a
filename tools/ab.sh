#!/bin/bash
# Interleaved A/B of an env switch on the config-3 bench (one process per run, same box).
# The release libyoda.so ignores the YODA_* tuning knobs: this runs the A/B build
# (make -C kubernetes-scheduler_amd/csrc ab -> libyoda_ab.so), which reads them.
#   usage: tools/ab.sh VAR "valA valB" [rounds]
set -o pipefail
VAR=$1; VALS=$2; R=${3:-3}
mkdir -p gpurun_out
for r in $(seq $R); do
  for v in $VALS; do
    env YODA_LIB_PATH=$(realpath kubernetes-scheduler_amd/yoda_amd/libyoda_ab.so) $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 \
      > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$VAR=$v', round(d['ms_per_step'],3), 'ms  k1', round(d['roofline']['k1_avg_ms'],3), 'k2', round(d['roofline']['k2_avg_ms'],3))"
  done
done
