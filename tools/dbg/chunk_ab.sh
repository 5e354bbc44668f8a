# Per-rank pod-shard step times under chunk-planning knobs (yoda_capi.cpp plan_chunks_for).
set -o pipefail
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u tools/pod_shard_timing.py --worlds 1,8 --kinds key256 || exit 1; }
{
run YODA_CHUNK_ROUNDS=6
run YODA_CHUNK_ROUNDS=3
run YODA_CHUNK_ROUNDS=2
run YODA_MIN_CHUNK_NODES=1024
run YODA_MIN_CHUNK_NODES=2048
run YODA_MIN_CHUNK_NODES=1024 YODA_CHUNK_ROUNDS=3
} > gpurun_out/chunk_ab.txt 2>&1
