#!/bin/bash
# Per-rank window kernels of the sharded greedy at 8 ranks (12.5k nodes each), rehearsed on one
# GPU (8 handles, in-process transport): rocprofv3 kernel trace of the windows alone, one run
# per flag, summarised (tools/kernel_trace_sum.py) and the raw trace deleted, for the DESIGN.md
# §7 latency model (each handle's kernels are what its rank would run).
#   usage (through gpurun): bash tools/greedy_rank_probe.sh <outdir> [flags...]
set -o pipefail
O=$(realpath -m $1); shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
for f in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $O/t$f -o run --output-format csv -- \
    python3 $R/tools/greedy_rehearsal.py --worlds 8 --no-single --flags $f > $O/rehearsal_$f.jsonl 2> $O/rehearsal_$f.err) || exit 1
  python3 $R/tools/kernel_trace_sum.py $(find $O/t$f -name "*kernel_trace.csv" | head -1) > $O/kernels_$f.json || exit 1
  rm -rf $O/t$f
done
