#!/bin/bash
# GPU pass after a kernel change: greedy tests, the greedy bench, and the rocprofv3 passes of
# the headline bench (tools/profile.sh) into gpurun_out/prof.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_greedy_config5.py \
  tests/test_gpu_greedy_sharded.py -k greedy -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_greedy.log 2>&1 || { tail -30 gpurun_out/pytest_greedy.log; exit 1; }
tail -2 gpurun_out/pytest_greedy.log
timeout -k 10 400 python bench.py --workload greedy > gpurun_out/bench_greedy.json 2> gpurun_out/bench_greedy.err || { tail -20 gpurun_out/bench_greedy.err; exit 1; }
cat gpurun_out/bench_greedy.json
rm -rf gpurun_out/prof
timeout -k 10 600 bash tools/profile.sh gpurun_out/prof --steps 4 --warmup 1 --no-extras || exit 1
echo profile done
