set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/greedy_prof.py --flags 1 0 || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/gprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/gprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/greedy_prof.py --flags 1 > $GRAFT_REPO_ROOT/gpurun_out/gprof.log 2>&1 || exit 1
