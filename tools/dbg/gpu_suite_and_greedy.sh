#!/bin/bash
# Full GPU test suite, then the greedy bench (config 5) without the CPU baseline.
set -o pipefail
mkdir -p gpurun_out/suite
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --durations=8 > gpurun_out/suite/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/suite/pytest_gpu.log; exit 1; }
tail -12 gpurun_out/suite/pytest_gpu.log
timeout -k 10 200 python bench.py --workload greedy --no-cpu-baseline > gpurun_out/suite/bench_greedy.json 2> gpurun_out/suite/bench_greedy.err || { tail -20 gpurun_out/suite/bench_greedy.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/suite/bench_greedy.json'))
print(round(d['seconds'],3), d['windows'], d['exact_fallback_pods'], {k: round(v) for k, v in d['host_times_ms'].items()}, 'cap', round(d['capacity']['seconds'],3), d['capacity']['windows'], {k: round(v) for k, v in d['capacity']['host_times_ms'].items()})"
