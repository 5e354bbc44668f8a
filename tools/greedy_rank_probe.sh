#!/bin/bash
# Per-rank window kernels of the sharded greedy at 8 ranks (12.5k nodes each), rehearsed on one
# GPU (8 handles, in-process transport): rocprofv3 kernel trace of the windows alone, for the
# DESIGN.md §7 latency model (each handle's kernels are what its rank would run).
#   usage (through gpurun): bash tools/greedy_rank_probe.sh <outdir> [flags...]
set -o pipefail
O=$(realpath -m $1); shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- \
  python3 $R/tools/greedy_rehearsal.py --worlds 8 --no-single --flags "$@" > $O/rehearsal.jsonl 2> $O/rehearsal.err
