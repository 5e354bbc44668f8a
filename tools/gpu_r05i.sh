#!/bin/bash
# Chunk-mask A/B (YODA_CMASK=0: every (wave, chunk) writes its partials) + GPU tests + PMC.
set -o pipefail
O=gpurun_out/r05i; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 600 bash tools/ab_run.sh 3 "cm1|abl/cur.so|" "cm0|abl/cur.so|YODA_CMASK=0" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
for lab in cm1 cm0; do
  e=""; [ $lab = cm0 ] && e="YODA_CMASK=0"
  env YODA_LIB_PATH=$(realpath abl/cur.so) $e timeout -k 10 400 bash tools/profile.sh $O/prof_$lab --no-extras --steps 10 --warmup 2 || { tail -5 $O/prof_$lab/*.log; exit 1; }
  python3 tools/pmc_brief.py $O/prof_$lab/pmc_summary.json > $O/pmc_$lab.txt 2>&1 || true
  find $O/prof_$lab -name '*.csv' ! -name '*stats*' -delete
done
cat $O/pmc_cm1.txt $O/pmc_cm0.txt | cut -c1-200
