#!/bin/bash
# A/B of YODA_MIN_CHUNK_NODES on the greedy bench (config 5, one GPU).
set -o pipefail
OUT=gpurun_out/greedy_minchunk
mkdir -p $OUT
for m in ${MINCHUNKS:-0 256 512 1024 2048}; do
  YODA_MIN_CHUNK_NODES=$m timeout -k 10 120 python bench.py --workload greedy \
    --no-cpu-baseline > $OUT/m$m.json 2> $OUT/m$m.err || { tail -5 $OUT/m$m.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('$OUT/m$m.json'))
print('minchunk $m', round(d['seconds'],3), d['windows'], d['host_times_ms'], 'cap', round(d['capacity']['seconds'],3), d['capacity']['windows'], d['capacity']['host_times_ms'])"
done
