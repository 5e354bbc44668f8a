#!/bin/bash
# One gpurun call's GPU steps, each under its own time limit, outputs in gpurun_out/<tag>/.
# A step that fails ordinarily (a red test, a non-zero exit) is recorded and the next step runs;
# a step that crashes or times out (exit 124, 134, 137, 139) ends the session -- no retries.
#
#   tools/gpu_session.sh <tag> <step>...
#     tests                 the whole -m gpu suite
#     test:<pytest args>    e.g. "test:tests/test_gpu_shard_seeds.py -k comm"
#     bench                 bench.py --steps 20 --warmup 5 (the driver's command shape)
#     bench:<args>          bench.py with these arguments
#     profile               tools/profile.sh: kernel trace + the PMC passes (no extras)
#     variants:<names>      tools/variants.py <names> --steps 5
#     cmd:<command>         any command (python3 tools/..., rocprofv3 ...)
#   env: LIB=<path>         run every step against another libyoda build (YODA_LIB_PATH)
#        LIMIT=<seconds>    per-step time limit (default 400)
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
[ -n "$LIB" ] && export YODA_LIB_PATH=$(realpath "$LIB")
LIMIT=${LIMIT:-400}
i=0
for step in "$@"; do
  i=$((i + 1))
  name="$i.${step%%:*}"
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  echo "[$(date +%T)] step $name: $step" | tee -a "$O/session.txt"
  case "${step%%:*}" in
    tests) cmd="python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" ;;
    test) cmd="python3 -u -m pytest $arg -m gpu -q --timeout 300 --timeout-method thread" ;;
    bench) cmd="python3 -u bench.py ${arg:---steps 20 --warmup 5}" ;;
    profile) cmd="bash tools/profile.sh $ROOT/$O/prof --no-extras --steps 10 --warmup 3" ;;
    variants) cmd="python3 -u tools/variants.py ${arg//,/ } --steps 5" ;;
    cmd) cmd="$arg" ;;
    *) echo "unknown step $step" | tee -a "$O/session.txt"; exit 2 ;;
  esac
  timeout -k 10 "$LIMIT" bash -c "$cmd" > "$O/$name.out" 2> "$O/$name.err"
  rc=$?
  echo "[$(date +%T)] step $name rc=$rc" | tee -a "$O/session.txt"
  tail -3 "$O/$name.out" | cut -c1-400
  case $rc in
    124|134|137|139) echo "step $name crashed or timed out (rc $rc): session ends" | tee -a "$O/session.txt"
                     tail -20 "$O/$name.err"; exit $rc ;;
  esac
done
