#!/bin/bash
# Config-3 step time under chunk-round settings (YODA_CHUNK_ROUNDS1 / 2), two runs each.
set -o pipefail
mkdir -p gpurun_out/rounds3
for r in "6 8" "4 8" "8 8" "6 6" "6 10" "6 12"; do
  set -- $r
  for i in 1 2; do
    YODA_CHUNK_ROUNDS1=$1 YODA_CHUNK_ROUNDS2=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras > gpurun_out/rounds3/r.json 2> gpurun_out/rounds3/r.err || { tail -5 gpurun_out/rounds3/r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/rounds3/r.json')); r=d['roofline']
print('rounds $1 $2', round(d['ms_per_step'],4), 'k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4))"
  done
done
