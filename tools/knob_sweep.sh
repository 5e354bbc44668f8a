#!/bin/bash
# Step time of bench.py on the A/B build (libyoda_ab.so reads the YODA_* knobs) for a list of
# knob settings and pod counts, one process per run:
#   tools/knob_sweep.sh "ENV=a ENV2=b|ENV=c|..." "100000 12500" [rounds]
# ("-" = no knob).  --pods P < 100000 approximates one rank of a P-pod shard (same generator).
set -o pipefail
SETS=$1; PODS=${2:-100000}; R=${3:-1}
AB=$(realpath kubernetes-scheduler_amd/yoda_amd/libyoda_ab.so)
mkdir -p gpurun_out
for r in $(seq $R); do
  for p in $PODS; do
    IFS='|' read -ra S <<< "$SETS"
    for set in "${S[@]}"; do
      envs=""; [ "$set" != "-" ] && envs="$set"
      env YODA_LIB_PATH=$AB $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras \
        --steps 10 --warmup 3 --pods $p > gpurun_out/ks.json 2> gpurun_out/ks.err || { tail -5 gpurun_out/ks.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ks.json').read().strip().splitlines()[-1]); r=d['roofline']; print('pods=$p', '$set', round(d['ms_per_step'],4), 'ms  k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4), flush=True)"
    done
  done
done
