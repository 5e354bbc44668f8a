#!/bin/bash
# Variant regressions (memory in bytes, mixed-model, config-4 generator): knob / build A/B.
set -o pipefail
O=gpurun_out/${TAG:-r05y}; rm -rf $O; mkdir -p $O
for spec in "cur|abl/cur.so|" "k1w7|abl/k1w7.so|" "cm0|abl/cur.so|YODA_CMASK=0" "seed0|abl/cur.so|YODA_SEEDS=0" "lv0|abl/cur.so|YODA_KB_LEVELS=0" "dec0|abl/cur.so|YODA_KB_DEC=0" "gb0|abl/cur.so|YODA_GBEST=0" "z0|abl/cur.so|YODA_NODE_ZORDER=0" "side0|abl/cur.so|YODA_SIDE_COPY=0"; do
  IFS='|' read -r lab lib envs <<< "$spec"
  env YODA_LIB_PATH=$(realpath $lib) $envs timeout -k 10 300 python3 tools/variants.py bytes mixed50 het100k c4 --steps 5 > $O/v_$lab.jsonl 2> $O/v_$lab.err || { tail -5 $O/v_$lab.err; exit 1; }
  echo "$lab $(python3 -c "
import json
for l in open('$O/v_$lab.jsonl'):
    d=json.loads(l); print(d['variant'], round(d['ms_per_step'],3), round(d['k1_ms'],3), round(d['k2_ms'],3), end=' | ')
")" | tee -a $O/ab.txt
done
