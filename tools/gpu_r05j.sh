#!/bin/bash
# Occupancy A/B: K1 at 6 / 5 waves per SIMD (no VGPR spills at 6), K2 at 4.
set -o pipefail
O=gpurun_out/r05j; rm -rf $O; mkdir -p $O
timeout -k 10 900 bash tools/ab_run.sh 3 "cur|abl/cur.so|" "k1w6|abl/k1w6.so|" "k1w5|abl/k1w5.so|" "k2w4|abl/k2w4.so|" "k1w6k2w4|abl/k1w6k2w4.so|" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
env YODA_LIB_PATH=$(realpath abl/k1w6.so) timeout -k 10 400 bash tools/profile.sh $O/prof_k1w6 --no-extras --steps 10 --warmup 2 || { tail -5 $O/prof_k1w6/*.log; exit 1; }
python3 tools/pmc_brief.py $O/prof_k1w6/pmc_summary.json > $O/pmc_k1w6.txt 2>&1 || true
find $O/prof_k1w6 -name '*.csv' ! -name '*stats*' -delete
head -4 $O/pmc_k1w6.txt | cut -c1-200
