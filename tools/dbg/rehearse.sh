set -o pipefail
export YODA_BENCH_SAME_DEVICE=1 YODA_DIST_BACKEND=gloo
for n in 2 3; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 3 --warmup 1 --pods 20000 --nodes 30000 --check --no-cpu-baseline > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err || { tail -30 gpurun_out/rehearse_$n.err; exit 1; }
cat gpurun_out/rehearse_$n.json
done
