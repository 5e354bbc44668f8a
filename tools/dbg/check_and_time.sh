#!/bin/bash
# GPU suite, then the headline bench twice (no extras, no CPU baseline) and the greedy bench.
set -o pipefail
mkdir -p gpurun_out/ct
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ct/pytest.log 2>&1 || { tail -30 gpurun_out/ct/pytest.log; exit 1; }
tail -1 gpurun_out/ct/pytest.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras > gpurun_out/ct/b$i.json 2> gpurun_out/ct/b$i.err || { tail -5 gpurun_out/ct/b$i.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ct/b$i.json')); r=d['roofline']
print('config3', round(d['ms_per_step'],4), 'k1', round(r['k1_avg_ms'],4), 'k2', round(r['k2_avg_ms'],4))"
done
YODA_GREEDY_DEBUG=1 timeout -k 10 120 python bench.py --workload greedy --no-cpu-baseline > gpurun_out/ct/g.json 2> gpurun_out/ct/g.err || { tail -5 gpurun_out/ct/g.err; exit 1; }
grep "greedy" gpurun_out/ct/g.err | tail -3
python -c "
import json; d=json.load(open('gpurun_out/ct/g.json'))
print('greedy', round(d['seconds'],3), 'cap', round(d['capacity']['seconds'],3), d['capacity']['host_times_ms'])"
