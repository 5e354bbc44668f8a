#!/bin/bash
# Per-rank workloads of 4- and 8-way node sharding (100k pods x 25k / 12.5k nodes) under
# YODA_MIN_CHUNK_NODES (one process per setting; two runs each).
set -o pipefail
mkdir -p gpurun_out/mcr
for nn in 12500 25000; do
  for m in ${MINS:-0 1600 1560 700 3200}; do
    for i in 1 2; do
      YODA_MIN_CHUNK_NODES=$m timeout -k 10 120 python bench.py --nodes $nn --no-cpu-baseline --no-extras --steps 20 --warmup 3 > gpurun_out/mcr/b.json 2> gpurun_out/mcr/b.err || { tail -5 gpurun_out/mcr/b.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/mcr/b.json')); r=d['roofline']
print('nodes $nn min_chunk $m', round(d['ms_per_step'],4), 'k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4))"
    done
  done
done
