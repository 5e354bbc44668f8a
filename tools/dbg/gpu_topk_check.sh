set -o pipefail
mkdir -p gpurun_out/topk1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk.py tests/test_gpu_greedy_sharded.py "tests/test_gpu_parity.py" -k "topk or greedy" > gpurun_out/topk1/pytest.log 2>&1 || { tail -50 gpurun_out/topk1/pytest.log; exit 1; }
tail -3 gpurun_out/topk1/pytest.log
timeout -k 10 200 python bench.py --workload greedy --no-cpu-baseline > gpurun_out/topk1/bench_greedy.json 2> gpurun_out/topk1/bench_greedy.err || { tail -20 gpurun_out/topk1/bench_greedy.err; exit 1; }
cat gpurun_out/topk1/bench_greedy.json
