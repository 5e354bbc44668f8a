set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['roofline']['k2_avg_ms'], d['e2e_ms'])
print(json.dumps(d['extra']['classes']))
for k,v in d['extra']['variants'].items(): print(k, round(v['ms_per_step'],3), round(v['k1_ms'],3), round(v['k2_ms'],3))
print(json.dumps(d['extra']['plugin_row_latency']))
print(json.dumps(d['cpu_baseline'])[:600])"
