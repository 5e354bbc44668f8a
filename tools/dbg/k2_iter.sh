#!/bin/bash
# K2 iteration loop on the GPU box: parity tests, per-wave trace, headline bench (short).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_k2.log 2>&1 || { tail -30 gpurun_out/pytest_k2.log; exit 1; }
tail -2 gpurun_out/pytest_k2.log
YODA_K2_TRACE=40000 timeout -k 10 200 python tools/dbg/k2_classes.py > gpurun_out/trace.txt 2>&1 || { tail -20 gpurun_out/trace.txt; exit 1; }
tail -9 gpurun_out/trace.txt
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]);r=d['roofline']
print('k1', round(r['k1_avg_ms'],3), 'k2', round(r['k2_avg_ms'],3), 'step', round(d['ms_per_step'],3), 'value %.3e' % d['value'])"
