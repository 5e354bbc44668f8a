# Pod-shard checks on one GPU box: parity test, per-rank timing, N=2 rehearsal of both shardings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "pod_sharded or shard" > gpurun_out/pytest_podshard.log 2>&1 || { tail -30 gpurun_out/pytest_podshard.log; exit 1; }
tail -2 gpurun_out/pytest_podshard.log
timeout -k 10 400 python -u tools/pod_shard_timing.py > gpurun_out/pod_shard_timing.txt 2>&1 || { tail -20 gpurun_out/pod_shard_timing.txt; exit 1; }
cat gpurun_out/pod_shard_timing.txt
export YODA_BENCH_SAME_DEVICE=1 YODA_DIST_BACKEND=gloo
for s in pods nodes; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --shard $s --steps 3 --warmup 1 --pods 20000 --nodes 30000 --check --no-cpu-baseline > gpurun_out/rehearse_$s.json 2> gpurun_out/rehearse_$s.err || { tail -30 gpurun_out/rehearse_$s.err; exit 1; }
cat gpurun_out/rehearse_$s.json
done
