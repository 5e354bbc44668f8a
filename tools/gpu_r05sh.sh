#!/bin/bash
# Sharded capacity greedy with deep lists: greedy GPU tests + full-size rehearsal (world 2, 3).
set -o pipefail
O=gpurun_out/${TAG:-r05sh}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "greedy or comm" > $O/pytest_greedy.txt 2>&1 || { tail -30 $O/pytest_greedy.txt; exit 1; }
tail -1 $O/pytest_greedy.txt
timeout -k 10 700 python -u tools/greedy_rehearsal.py --worlds 2 3 > $O/greedy_rehearsal.jsonl 2> $O/greedy_rehearsal.err || { tail -20 $O/greedy_rehearsal.err; exit 1; }
cut -c1-330 $O/greedy_rehearsal.jsonl
