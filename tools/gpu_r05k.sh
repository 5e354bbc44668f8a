#!/bin/bash
# gbest publishing A/B: once per value (gpub) vs every refresh (repub) vs no shared best.
set -o pipefail
O=gpurun_out/r05k; rm -rf $O; mkdir -p $O
timeout -k 10 900 bash tools/ab_run.sh 3 "gpub|abl/gpub.so|" "repub|abl/repub.so|" "gb0|abl/gpub.so|YODA_GBEST=0" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
for spec in "gpub|abl/gpub.so|" "repub|abl/repub.so|" "gb0|abl/gpub.so|YODA_GBEST=0"; do
  IFS='|' read -r lab lib envs <<< "$spec"
  env YODA_LIB_PATH=$(realpath $lib) $envs timeout -k 10 400 bash tools/profile.sh $O/prof_$lab --no-extras --steps 10 --warmup 2 || { tail -5 $O/prof_$lab/*.log; exit 1; }
  python3 tools/pmc_brief.py $O/prof_$lab/pmc_summary.json > $O/pmc_$lab.txt 2>&1 || true
  find $O/prof_$lab -name '*.csv' ! -name '*stats*' -delete
  echo $lab; head -3 $O/pmc_$lab.txt | cut -c1-200
done
