#!/bin/bash
# Quick GPU pass: the -m gpu suite (optionally a -k filter), then tools/variants.py on the
# named workloads with a sampled oracle check.
#   usage (through gpurun): bash tools/gpu_quick.sh <outdir> "<pytest -k expr or ''>" variant...
set -o pipefail
O=$1; K=$2; shift 2
rm -rf $O && mkdir -p $O
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  "${KA[@]}" --durations=10 > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u tools/variants.py "$@" --steps 5 --check 128 > $O/variants.jsonl 2> $O/variants.err \
    || { tail -20 $O/variants.err; exit 1; }
  cut -c1-600 $O/variants.jsonl
fi
