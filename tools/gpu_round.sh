#!/bin/bash
# One GPU-box pass: parity tests, the headline bench, the greedy bench (config 5), and
# optionally the rocprofv3 passes.
#   usage: tools/gpu_round.sh [profile]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  --durations=15 > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 python bench.py --workload greedy > gpurun_out/bench_greedy.json 2> gpurun_out/bench_greedy.err || { tail -20 gpurun_out/bench_greedy.err; exit 1; }
cat gpurun_out/bench_greedy.json
if [ "$1" = "profile" ]; then
  timeout -k 10 600 bash tools/profile.sh gpurun_out/prof --steps 4 --warmup 1 --no-extras || exit 1
fi
