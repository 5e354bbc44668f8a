#!/bin/bash
# Deep lists with the early-exit resolve scan: greedy tests, depth A/B, kernel totals at 64.
set -o pipefail
O=gpurun_out/${TAG:-r05q}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "greedy" > $O/pytest_greedy.txt 2>&1 || { tail -30 $O/pytest_greedy.txt; exit 1; }
tail -1 $O/pytest_greedy.txt
for r in 1 2; do
  for d in 64; do
    echo "depth$d $(YODA_GREEDY_DEBUG=1 YODA_LIB_PATH=$(realpath abl/cur.so) YODA_GREEDY_CAP_DEPTH=$d timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 2>&1 | grep -E '^flags|restarts' | tail -2 | cut -c1-300 | tr '\n' ' ')" | tee -a $O/depth_ab.txt
  done
done
echo "dma0 $(YODA_GREEDY_DEBUG=1 YODA_LIB_PATH=$(realpath abl/cur.so) YODA_WIN_DMA=0 timeout -k 10 300 python3 tools/greedy_prof.py --flags 1 2>&1 | grep -E '^flags' | cut -c1-200)" | tee -a $O/depth_ab.txt
cd /tmp && export TMPDIR=/tmp
YODA_LIB_PATH=$GRAFT_REPO_ROOT/abl/cur.so YODA_GREEDY_CAP_DEPTH=64 YODA_GREEDY_TRACE=$GRAFT_REPO_ROOT/$O/windows64.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/greedy_prof.py --flags 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_trace_sum.py $T > $O/kernels64.json
find $O/prof -name '*kernel_trace.csv' -delete
awk '{n++; a+=$9; b+=$10; c+=$11; d+=$12; e+=$13; r+=$3; w+=$2} END {print n, "mean total",a/n,"up",b/n,"issued",c/n,"sync",d/n,"win",e/n, "resolved/win", r/n, "wn", w/n}' $O/windows64.txt
head -c 1200 $O/kernels64.json
