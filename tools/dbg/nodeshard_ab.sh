# Node-shard per-rank kernel time under chunk knobs at W=2,4,8, plus a kernel-trace profile at W=8.
set -o pipefail
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u tools/pod_shard_timing.py --worlds 2,4,8 --kinds nodes 2>&1 | grep -v amdgpu.ids || exit 1; }
{
run YODA_CHUNK_ROUNDS=6
run YODA_MIN_CHUNK_NODES=1024
run YODA_MIN_CHUNK_NODES=2048
run YODA_CHUNK_ROUNDS=3
run YODA_CHUNK_ROUNDS=12
} > gpurun_out/nodeshard_ab.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ns8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pod_shard_timing.py --worlds 8 --kinds nodes > $GRAFT_REPO_ROOT/gpurun_out/prof_ns8.log 2>&1
