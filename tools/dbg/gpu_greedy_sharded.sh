set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_greedy_sharded.py tests/test_gpu_parity.py -k "greedy or sharded" -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_greedy.log 2>&1 || { tail -60 gpurun_out/pytest_greedy.log; exit 1; }
tail -15 gpurun_out/pytest_greedy.log
YODA_BENCH_SAME_DEVICE=1 YODA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --workload greedy --gpus 2 --pods 100000 --check > gpurun_out/greedy2.json 2> gpurun_out/greedy2.err || { tail -30 gpurun_out/greedy2.err; exit 1; }
cat gpurun_out/greedy2.json
