#!/bin/bash
# Variant timings: the current build (non-G bounds gated to one-model K <= 8) and builds of
# earlier round-5 commits (memory-in-bytes regression bisect).
set -o pipefail
O=gpurun_out/${TAG:-r05z}; rm -rf $O; mkdir -p $O
for spec in "cur|kubernetes-scheduler_amd/yoda_amd/libyoda.so" "00bd14f|abl/at_00bd14f.so" "67b1550|abl/at_67b1550.so" "2401a02|abl/at_2401a02.so" "718338c|abl/at_718338c.so"; do
  IFS='|' read -r lab lib <<< "$spec"
  env YODA_LIB_PATH=$(realpath $lib) timeout -k 10 300 python3 tools/variants.py bytes mixed50 het100k c4 c3 --steps 5 > $O/v_$lab.jsonl 2> $O/v_$lab.err || { tail -5 $O/v_$lab.err; exit 1; }
  echo "$lab $(python3 -c "
import json
for l in open('$O/v_$lab.jsonl'):
    d=json.loads(l); print(d['variant'], round(d['ms_per_step'],3), round(d['k1_ms'],3), round(d['k2_ms'],3), end=' | ')
")" | tee -a $O/ab.txt
done
