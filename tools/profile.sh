#!/bin/bash
# Kernel-trace + PMC passes of bench.py on a GPU box (run through gpurun).  Each counter
# group gets its own rocprofv3 pass (MI355X_MICROARCH.md: TCC FETCH_SIZE and WRITE_SIZE do
# not fit one pass); only --kernel-trace is combined with --pmc.
#   usage: tools/profile.sh <outdir> [bench args...]
set -euo pipefail
OUT=$(realpath -m "$1"); shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@")
run() {  # name, extra rocprofv3 args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline "${ARGS[@]}" > "$OUT/$name.log" 2>&1
}
run trace --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
run sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run sq2 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/pmc_summary.json"
