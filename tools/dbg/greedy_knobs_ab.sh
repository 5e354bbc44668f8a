#!/bin/bash
# Greedy bench (config 5) under A/B knob settings: each argument is one "VAR=val VAR2=val" set.
set -o pipefail
OUT=gpurun_out/greedy_knobs
mkdir -p $OUT
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 120 python bench.py --workload greedy --no-cpu-baseline > $OUT/r$i.json 2> $OUT/r$i.err || { tail -5 $OUT/r$i.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('$OUT/r$i.json'))
print('[$kv]', round(d['seconds'],3), d['windows'], d['exact_fallback_pods'], {k: round(v) for k, v in d['host_times_ms'].items()}, 'cap', round(d['capacity']['seconds'],3), d['capacity']['windows'], {k: round(v) for k, v in d['capacity']['host_times_ms'].items()})"
done
