#!/bin/bash
# A/B of the chunk rounds (YODA_CHUNK_ROUNDS1/2) on the greedy bench (config 5, one GPU).
set -o pipefail
OUT=gpurun_out/greedy_rounds
mkdir -p $OUT
for r in "6 8" "2 2" "1 1" "1 2"; do
  set -- $r
  YODA_CHUNK_ROUNDS1=$1 YODA_CHUNK_ROUNDS2=$2 timeout -k 10 120 python bench.py --workload greedy \
    --no-cpu-baseline > $OUT/r$1_$2.json 2> $OUT/r$1_$2.err || { tail -5 $OUT/r$1_$2.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('$OUT/r$1_$2.json'))
print('rounds $1 $2', round(d['seconds'],3), d['host_times_ms'], 'cap', round(d['capacity']['seconds'],3), d['capacity']['host_times_ms'])"
done
