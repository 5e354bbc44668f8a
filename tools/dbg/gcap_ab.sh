#!/bin/bash
# A/B of the capacity greedy's fallback policy (YODA_GREEDY_FAIL_DIV) on config 5.
set -o pipefail
mkdir -p gpurun_out
for d in 0 64 32 8; do
  YODA_GREEDY_FAIL_DIV=$d YODA_GREEDY_DEBUG=1 timeout -k 10 300 python3 tools/dbg/greedy_capacity_dbg.py ${1:-1000000} >> gpurun_out/gcap_ab.log 2>&1 || exit 1
  echo "div=$d done" >> gpurun_out/gcap_ab.log
done
grep -v amdgpu.ids gpurun_out/gcap_ab.log
