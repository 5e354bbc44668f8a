set -o pipefail
mkdir -p gpurun_out/abv
for r in 1 2; do
  for spec in head:abx/head.so staged:kubernetes-scheduler_amd/yoda_amd/libyoda.so w6:abx/w6.so; do
    lab=${spec%%:*}; lib=${spec#*:}
    YODA_LIB_PATH=$(realpath $lib) timeout -k 10 120 python3 tools/variants.py c3 mixed50 mixed100 het100k c4 --steps 5 > gpurun_out/abv/$lab.$r.out 2> gpurun_out/abv/$lab.$r.err || exit 1
    python3 -c "
import json,sys
for l in open('gpurun_out/abv/$lab.$r.out'):
    if l.startswith('{'):
        d=json.loads(l); print('$lab', d['variant'], round(d['ms_per_step'],4), 'k1', round(d['k1_ms'],4), 'k2', round(d['k2_ms'],4))
"
  done
done
