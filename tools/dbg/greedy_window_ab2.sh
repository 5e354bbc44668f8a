#!/bin/bash
# A/B of YODA_GREEDY_WINDOW on the greedy bench (config 5, one GPU), block top-k K2.
set -o pipefail
OUT=gpurun_out/greedy_window2
mkdir -p $OUT
for w in ${WINDOWS:-4096 8192 16384 32768}; do
  YODA_GREEDY_WINDOW=$w timeout -k 10 120 python bench.py --workload greedy \
    --no-cpu-baseline > $OUT/w$w.json 2> $OUT/w$w.err || { tail -5 $OUT/w$w.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('$OUT/w$w.json'))
print('window $w', round(d['seconds'],3), d['windows'], d['exact_fallback_pods'], d['host_times_ms'], 'cap', round(d['capacity']['seconds'],3), d['capacity']['windows'])"
done
