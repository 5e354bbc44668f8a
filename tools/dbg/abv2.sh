set -o pipefail
mkdir -p gpurun_out/abv2
for r in 1 2; do
  for spec in "k2only-lpt0|abx/k2only.so|YODA_K1_LPT=0" "new-lpt0|abx/newab.so|YODA_K1_LPT=0" "new-lpt1|abx/newab.so|" "k2only-lpt1|abx/k2only.so|"; do
    IFS='|' read -r lab lib envs <<< "$spec"
    env YODA_LIB_PATH=$(realpath $lib) $envs timeout -k 10 120 python3 tools/variants.py mixed50 --steps 5 > gpurun_out/abv2/$lab.$r.out 2> gpurun_out/abv2/$lab.$r.err || exit 1
    python3 -c "
import json,sys
for l in open('gpurun_out/abv2/$lab.$r.out'):
    if l.startswith('{'):
        d=json.loads(l); print('$lab', d['variant'], round(d['ms_per_step'],4), 'k1', round(d['k1_ms'],4), 'k2', round(d['k2_ms'],4), d['classes']['k1_blocks'])
"
  done
done
