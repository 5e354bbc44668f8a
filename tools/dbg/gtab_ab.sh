#!/bin/bash
# G-table A/B on the headline bench (config 3) + the GPU parity suite.
set -o pipefail
mkdir -p gpurun_out/gtab
if [ -z "$SKIP_TESTS" ]; then timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gtab/pytest.log 2>&1 || { tail -30 gpurun_out/gtab/pytest.log; exit 1; }; fi
tail -2 gpurun_out/gtab/pytest.log
for v in ${GTAB_VARIANTS:-0 1 0 1}; do
  YODA_NO_GTAB=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras > gpurun_out/gtab/b$v.json 2> gpurun_out/gtab/b$v.err || { tail -5 gpurun_out/gtab/b$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/gtab/b$v.json')); r=d['roofline']
print('NO_GTAB=$v', round(d['ms_per_step'],4), 'k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4))"
done
