#!/bin/bash
# Round-4 final GPU pass into gpurun_out/final: the -m gpu suite, the headline bench (extras and
# CPU baseline), the rocprofv3 kernel-trace + PMC passes of it, the greedy bench (config 5,
# both flags) and the one-GPU sharded greedy rehearsal (world 2 and 3).
set -o pipefail
O=gpurun_out/final
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  --durations=20 > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
timeout -k 10 700 bash tools/profile.sh $O/prof --steps 4 --warmup 1 --no-extras > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 tools/pmc_brief.py $O/prof/pmc_summary.json | head -8
timeout -k 10 400 python bench.py --workload greedy > $O/bench_greedy.json 2> $O/bench_greedy.err || { tail -20 $O/bench_greedy.err; exit 1; }
cut -c1-800 $O/bench_greedy.json
timeout -k 10 600 python -u tools/greedy_rehearsal.py --worlds 2 3 > $O/greedy_rehearsal.jsonl 2> $O/greedy_rehearsal.err || { tail -20 $O/greedy_rehearsal.err; exit 1; }
cat $O/greedy_rehearsal.jsonl
