set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/pod_shard_timing.py --worlds 4,8 --kinds nodes --all-ranks > gpurun_out/balance.txt 2>&1 || { tail -20 gpurun_out/balance.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/balance.txt
export YODA_BENCH_SAME_DEVICE=1 YODA_DIST_BACKEND=gloo
for n in 2 3; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 3 --warmup 1 --pods 20000 --nodes 30000 --check --no-cpu-baseline > gpurun_out/rehearse_bal_$n.json 2> gpurun_out/rehearse_bal_$n.err || { tail -30 gpurun_out/rehearse_bal_$n.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/rehearse_bal_$n.json').read().strip().splitlines()[-1]); print('$n', d['config']['parallelism'], d['config']['node_bounds'], d.get('check'))"
done
