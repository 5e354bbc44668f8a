#!/bin/bash
# One GPU-box pass: parity tests, then the bench (and optionally the rocprofv3 passes).
#   usage: tools/gpu_round.sh [profile]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ "$1" = "profile" ]; then
  timeout -k 10 600 bash tools/profile.sh gpurun_out/prof --steps 4 --warmup 1 || exit 1
fi
