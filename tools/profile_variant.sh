#!/bin/bash
# rocprofv3 passes of tools/variants.py on a GPU box (through gpurun): a kernel trace with
# stats, then one counter group per pass (MI355X_MICROARCH.md: one block's counters per pass).
#   usage: tools/profile_variant.sh <outdir> <variant> [more variants...]
set -euo pipefail
OUT=$(realpath -m "$1"); shift
VARGS=("$@")
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv \
    -- python3 "$ROOT/tools/variants.py" "${VARGS[@]}" --steps 3 > "$OUT/$name.log" 2>&1
}
run trace --kernel-trace --stats
run sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run sq2 --kernel-trace --pmc SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/pmc_summary.json"
