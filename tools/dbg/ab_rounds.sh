#!/bin/bash
# A/B of the chunk rounds used for small batches (greedy windows): config 5 greedy bench.
set -o pipefail
mkdir -p gpurun_out
for r in 6 2 1 3 6 2; do
  YODA_SMALL_ROUNDS=$r timeout -k 10 200 python bench.py --workload greedy --no-cpu-baseline > gpurun_out/ab_r$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_r$r.json'));print($r, round(d['seconds'],4), d['host_times_ms'], d['exact_fallback_pods'])"
done
