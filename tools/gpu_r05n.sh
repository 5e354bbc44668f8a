#!/bin/bash
# GPU suite + e2e split (side copy + pinned picks download) + a default bench line.
set -o pipefail
O=gpurun_out/r05n; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for r in 1 2 3; do YODA_UPLOAD_DEBUG=1 timeout -k 10 200 python3 tools/dbg/e2e_split.py 2>&1 | tail -2 | tee -a $O/e2e_split.txt || exit 1; done
timeout -k 10 300 python bench.py --no-extras > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('e2e_ms'), d['roofline'].get('k2_avg_ms'))"
for r in 1 2; do
  for v in 1 0; do
    echo "owncap$v $(YODA_LIB_PATH=$(realpath abl/cur.so) YODA_TOPK_OWN_CAP=$v timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 0 2>&1 | grep '^flags' | cut -c1-60 | tr '\n' ' ')" | tee -a $O/greedy_owncap_ab.txt
  done
done
YODA_UPLOAD_DEBUG=1 timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 > $O/greedy_updbg.out 2> $O/greedy_updbg.err || { tail -3 $O/greedy_updbg.err; exit 1; }
python3 - $O/greedy_updbg.err <<'PY'
import re, sys
v = [list(map(float, m.groups())) for m in (re.search(r"pack ([\d.]+) merge ([\d.]+) copy ([\d.]+) groups ([\d.]+)", l) for l in open(sys.argv[1])) if m]
n = len(v)
print("uploads", n, "mean pack/merge/copy/groups ms", [round(sum(x[i] for x in v) / n, 4) for i in range(4)])
PY
rm -f $O/greedy_updbg.err
