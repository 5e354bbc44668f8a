# Full GPU parity suite, N=2/3 rehearsals of both shardings (gloo, one GPU), then the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
export YODA_BENCH_SAME_DEVICE=1 YODA_DIST_BACKEND=gloo
for n in 2 3; do for s in nodes pods; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --shard $s --steps 3 --warmup 1 --pods 20000 --nodes 30000 --check --no-cpu-baseline > gpurun_out/rehearse_${s}_$n.json 2> gpurun_out/rehearse_${s}_$n.err || { tail -30 gpurun_out/rehearse_${s}_$n.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/rehearse_${s}_$n.json').read().strip().splitlines()[-1]); print('$s $n', d['config']['parallelism'], d.get('check'))"
done; done
unset YODA_BENCH_SAME_DEVICE YODA_DIST_BACKEND
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-400 gpurun_out/bench.json
