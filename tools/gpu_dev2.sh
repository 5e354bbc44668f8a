#!/bin/bash
# GPU pass: the -m gpu suite, the headline bench + its rocprofv3 passes, and a kernel trace of
# the capacity greedy batch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --no-extras > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-1200 gpurun_out/bench.json
rm -rf gpurun_out/prof gpurun_out/gprof
timeout -k 10 600 bash tools/profile.sh gpurun_out/prof --steps 4 --warmup 1 --no-extras || exit 1
python3 tools/pmc_brief.py gpurun_out/prof/pmc_summary.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/gprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/greedy_prof.py --flags 1 0 > $GRAFT_REPO_ROOT/gpurun_out/gprof.log 2>&1 || exit 1
cat $GRAFT_REPO_ROOT/gpurun_out/gprof.log | tail -3
