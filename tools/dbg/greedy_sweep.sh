#!/bin/bash
# Config-5 greedy seconds (flags 0 / capacity) on the A/B build for a list of knob settings:
#   tools/dbg/greedy_sweep.sh "-|YODA_GREEDY_CAP_DEPTH=96|..." [rounds]
set -o pipefail
SETS=$1; R=${2:-1}
AB=$(realpath kubernetes-scheduler_amd/yoda_amd/libyoda_ab.so)
mkdir -p gpurun_out
for r in $(seq $R); do
  IFS='|' read -ra S <<< "$SETS"
  for set in "${S[@]}"; do
    envs=""; [ "$set" != "-" ] && envs="$set"
    env YODA_LIB_PATH=$AB $envs timeout -k 10 300 python3 bench.py --workload greedy --steps 1 --warmup 0 \
      --no-cpu-baseline > gpurun_out/gs.json 2> gpurun_out/gs.err || { tail -5 gpurun_out/gs.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/gs.json').read().strip().splitlines()[-1]); c=d['capacity']; print('$set', round(d['seconds'],4), 's  capacity', round(c['seconds'],4), 's windows', c.get('windows'), 'restarts', c.get('window_restarts'), flush=True)"
  done
done
