#!/bin/bash
# Development GPU pass: the -m gpu suite (optional -k filter), the headline bench (with class
# counters) and the greedy bench.   usage: tools/gpu_dev.sh "<pytest -k expr or ''>" [greedy]
set -o pipefail
mkdir -p gpurun_out
K=$1
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  "${KA[@]}" --durations=15 > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-3000 gpurun_out/bench.json
if [ "$2" = "greedy" ]; then
  timeout -k 10 400 python bench.py --workload greedy > gpurun_out/bench_greedy.json 2> gpurun_out/bench_greedy.err || { tail -20 gpurun_out/bench_greedy.err; exit 1; }
  cut -c1-3000 gpurun_out/bench_greedy.json
fi
