set -o pipefail
mkdir -p gpurun_out
{
timeout -k 10 200 python -u tools/pod_shard_timing.py --worlds 8 --kinds key256,snake256,key64 || exit 1
timeout -k 10 200 python -u tools/pod_shard_timing.py --worlds 8 --kinds key256 --reverse || exit 1
} > gpurun_out/deal_ab.txt 2>&1
