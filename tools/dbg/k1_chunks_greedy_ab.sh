#!/bin/bash
# A/B of the K1 chunk cap (YODA_K1_MAX_CHUNKS) on the config-5 greedy bench (both flags).
set -o pipefail
mkdir -p gpurun_out/k1c
for c in 0 784 392 196; do
  if [ "$c" = 0 ]; then unset YODA_K1_MAX_CHUNKS; else export YODA_K1_MAX_CHUNKS=$c; fi
  timeout -k 10 150 python bench.py --workload greedy --no-cpu-baseline > gpurun_out/k1c/g$c.json 2> gpurun_out/k1c/g$c.err || { tail -5 gpurun_out/k1c/g$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/k1c/g$c.json'))
print('max_chunks $c', 'greedy', round(d['seconds'],3), 'cap', round(d['capacity']['seconds'],3), round(d['capacity']['host_times_ms']['window_ms'],1))"
done
