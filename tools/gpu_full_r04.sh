#!/bin/bash
# Full GPU pass: the whole -m gpu suite (every-pick full-size digests included), the greedy
# bench (config 5, both flags) and the one-GPU sharded greedy rehearsal (world 2 and 3).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  --durations=20 > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --workload greedy > gpurun_out/bench_greedy.json 2> gpurun_out/bench_greedy.err || { tail -20 gpurun_out/bench_greedy.err; exit 1; }
cut -c1-2500 gpurun_out/bench_greedy.json
timeout -k 10 600 python -u tools/greedy_rehearsal.py --worlds 2 3 > gpurun_out/greedy_rehearsal.jsonl 2> gpurun_out/greedy_rehearsal.err || { tail -20 gpurun_out/greedy_rehearsal.err; exit 1; }
cat gpurun_out/greedy_rehearsal.jsonl
