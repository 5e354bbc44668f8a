#!/bin/bash
# Step time of the release libyoda at several pod counts (one pod-sharded rank's batch):
#   tools/dbg/pods_probe.sh "100000 50000 25000 12500"
set -o pipefail
mkdir -p gpurun_out
for p in $1; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 --pods $p \
    > gpurun_out/pp.json 2> gpurun_out/pp.err || { tail -5 gpurun_out/pp.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/pp.json').read().strip().splitlines()[-1]); r=d['roofline']; print('pods=$p', round(d['ms_per_step'],4), 'ms  k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4), flush=True)"
done
