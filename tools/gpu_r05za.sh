#!/bin/bash
# Full GPU suite + variant timings of the current build.
set -o pipefail
O=gpurun_out/${TAG:-r05za}; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python3 tools/variants.py bytes mixed50 het100k c4 c3 --steps 5 > $O/v.jsonl 2> $O/v.err || { tail -5 $O/v.err; exit 1; }
python3 -c "
import json
for l in open('$O/v.jsonl'):
    d=json.loads(l); print(d['variant'], round(d['ms_per_step'],3), round(d['k1_ms'],3), round(d['k2_ms'],3), end=' | ')
"
