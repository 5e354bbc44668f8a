#!/bin/bash
# Interleaved A/B runs of the config-3 bench, one process per run, same box:
#   tools/ab_run.sh <rounds> "<label>|<lib .so>|<env assignments>" ...
# prints "<label> ms/step k1 k2" per run (HIP-event K1 / K2 ms).
set -o pipefail
R=$1; shift
mkdir -p gpurun_out
for r in $(seq $R); do
  for spec in "$@"; do
    IFS='|' read -r lab lib envs <<< "$spec"
    env YODA_LIB_PATH=$(realpath $lib) $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras \
      --steps 10 --warmup 2 > gpurun_out/ab_$lab.json 2> gpurun_out/ab_$lab.err || { tail -5 gpurun_out/ab_$lab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['ms_per_step'],4), 'k1', round(d['roofline']['k1_avg_ms'],4), 'k2', round(d['roofline']['k2_avg_ms'],4))"
  done
done
