#!/bin/bash
# Headline bench (config 3) under several environment settings, interleaved, one box.
#   usage: tools/dbg/bench_env_ab.sh "VAR=a VAR=b ..." [rounds]   (each word: one run's env)
set -o pipefail
for r in $(seq ${2:-2}); do
  for e in $1; do
    echo -n "$e: "
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4))" || exit 1
  done
done
