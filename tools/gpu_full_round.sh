#!/bin/bash
# One complete GPU pass for the round record: the -m gpu suite, the rocprofv3 kernel-trace +
# PMC passes of the headline bench (tools/profile.sh), then the headline bench (extras + CPU
# baseline, reading the fresh PMC summary) and the greedy bench (config 5).
#   usage (through gpurun): bash tools/gpu_full_round.sh
set -o pipefail
O=gpurun_out/full
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --durations=15 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 bash tools/profile.sh $O/prof --steps 4 --warmup 1 --no-extras || { echo profile failed; exit 1; }
cp $O/prof/pmc_summary.json profiles/pmc_latest.json
find $O/prof/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python bench.py --workload greedy > $O/bench_greedy.json 2> $O/bench_greedy.err || { tail -20 $O/bench_greedy.err; exit 1; }
cat $O/bench_greedy.json
