#!/bin/bash
# Round-5 GPU pass into gpurun_out/<tag>: the -m gpu suite, the headline bench (extras and CPU
# baseline), the end-to-end split (upload / run / download), the greedy bench (config 5, both
# flags), optionally the rocprofv3 kernel-trace + PMC passes (PROF=1).
#   usage (through gpurun): bash tools/gpu_r05.sh <tag> [pytest -k expr]
set -o pipefail
O=gpurun_out/$1; K=$2
rm -rf $O && mkdir -p $O
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  "${KA[@]}" --durations=15 > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  cut -c1-700 $O/bench.json
  YODA_UPLOAD_DEBUG=1 timeout -k 10 200 python tools/dbg/e2e_split.py > $O/e2e_split.txt 2>&1 || { tail -20 $O/e2e_split.txt; exit 1; }
  tail -3 $O/e2e_split.txt
fi
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 700 bash tools/profile.sh $O/prof --steps 4 --warmup 1 --no-extras > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
  python3 tools/pmc_brief.py $O/prof/pmc_summary.json | head -12
fi
if [ "${GREEDY:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py --workload greedy > $O/bench_greedy.json 2> $O/bench_greedy.err || { tail -20 $O/bench_greedy.err; exit 1; }
  cut -c1-900 $O/bench_greedy.json
fi
if [ "${REHEARSE:-0}" = 1 ]; then
  timeout -k 10 600 python -u tools/greedy_rehearsal.py --worlds 2 3 > $O/greedy_rehearsal.jsonl 2> $O/greedy_rehearsal.err || { tail -20 $O/greedy_rehearsal.err; exit 1; }
  cut -c1-400 $O/greedy_rehearsal.jsonl
fi
