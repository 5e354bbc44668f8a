#!/bin/bash
# N = 2 rehearsals of the multi-GPU bench on ONE GPU (gloo transport, both ranks on device 0):
# node sharding with --check (merged picks == a single handle), the libyoda exchange, and the
# sharded greedy with --check.  Prints the JSON lines.
set -o pipefail
export YODA_BENCH_SAME_DEVICE=1 YODA_DIST_BACKEND=gloo
mkdir -p gpurun_out/reh
run() {
  local name=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29513 bench.py --gpus 2 "$@" > gpurun_out/reh/$name.json 2> gpurun_out/reh/$name.err || { tail -30 gpurun_out/reh/$name.err; exit 1; }
  head -c 600 gpurun_out/reh/$name.json; echo
}
run nodes --steps 3 --warmup 1 --check --no-cpu-baseline
run greedy --workload greedy --pods 200000 --check --no-cpu-baseline
