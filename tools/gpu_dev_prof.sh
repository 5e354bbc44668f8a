#!/bin/bash
# Development GPU pass with profiles: the -m gpu suite (optional -k filter), the headline
# bench, and the rocprofv3 kernel-trace + PMC passes of it (tools/profile.sh) into
# gpurun_out/prof.   usage: tools/gpu_dev_prof.sh "<pytest -k expr or ''>"
set -o pipefail
mkdir -p gpurun_out
K=$1
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  "${KA[@]}" --durations=15 > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-1500 gpurun_out/bench.json
rm -rf gpurun_out/prof
timeout -k 10 600 bash tools/profile.sh gpurun_out/prof --steps 4 --warmup 1 --no-extras || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/prof/pmc_summary.json'));print(json.dumps({k:v for k,v in d.items() if k in ('k1_block_n32','k2_block_n32','k_reduce1','k_reduce2')})[:3000])"
