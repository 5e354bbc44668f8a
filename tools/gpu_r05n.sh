#!/bin/bash
# GPU suite + e2e split (side copy + pinned picks download) + a default bench line.
set -o pipefail
O=gpurun_out/r05n; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for r in 1 2 3; do timeout -k 10 200 python3 tools/dbg/e2e_split.py 2>&1 | tail -1 | tee -a $O/e2e_split.txt || exit 1; done
timeout -k 10 300 python bench.py --no-extras > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('e2e_ms'), d['roofline'].get('k2_avg_ms'))"
