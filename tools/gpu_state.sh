#!/bin/bash
# State pass on a GPU box: the -m gpu suite, every tools/variants.py workload (with a sampled
# oracle check), and the greedy bench (config 5).
#   usage (through gpurun): bash tools/gpu_state.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/state}
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --durations=15 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u tools/variants.py --steps 5 --check 128 > $O/variants.jsonl 2> $O/variants.err \
  || { tail -20 $O/variants.err; exit 1; }
cut -c1-400 $O/variants.jsonl
timeout -k 10 400 python bench.py --workload greedy > $O/bench_greedy.json 2> $O/bench_greedy.err \
  || { tail -20 $O/bench_greedy.err; exit 1; }
cat $O/bench_greedy.json
