#!/bin/bash
# One 8-way node-shard rank's workload (100k pods x 12.5k nodes) under YODA_MIN_CHUNK_NODES.
set -o pipefail
mkdir -p gpurun_out/mc8
for m in ${MINS:-0 780 1560 3125}; do
  for i in 1 2; do
    YODA_MIN_CHUNK_NODES=$m timeout -k 10 120 python bench.py --nodes 12500 --no-cpu-baseline --no-extras --steps 20 --warmup 3 > gpurun_out/mc8/b.json 2> gpurun_out/mc8/b.err || { tail -5 gpurun_out/mc8/b.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/mc8/b.json')); r=d['roofline']
print('min_chunk $m', round(d['ms_per_step'],4), 'k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4))"
  done
done
