#!/bin/bash
# K2 write traffic at 4 waves per SIMD (no VGPR spills) vs the default 5: PMC passes.
set -o pipefail
O=gpurun_out/r05k2w; rm -rf $O; mkdir -p $O
env YODA_LIB_PATH=$(realpath abl/k2w4.so) timeout -k 10 400 bash tools/profile.sh $O/prof_k2w4 --no-extras --steps 10 --warmup 2 || { tail -5 $O/prof_k2w4/*.log; exit 1; }
python3 tools/pmc_brief.py $O/prof_k2w4/pmc_summary.json > $O/pmc_k2w4.txt 2>&1 || true
find $O/prof_k2w4 -name '*.csv' ! -name '*stats*' -delete
head -3 $O/pmc_k2w4.txt | cut -c1-200
