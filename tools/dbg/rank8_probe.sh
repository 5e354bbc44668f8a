set -o pipefail
mkdir -p gpurun_out/r8
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r8/t -o run --output-format csv -- python3 $R/bench.py --nodes 12500 --no-cpu-baseline --no-extras --steps 20 --warmup 3 > $R/gpurun_out/r8/b.json 2> $R/gpurun_out/r8/b.err
cd $R
python3 -c "
import json; d=json.load(open('gpurun_out/r8/b.json')); print('ms_per_step', d['ms_per_step'])"
python3 tools/dbg/greedy_kernel_split.py gpurun_out/r8/t/run_kernel_trace.csv
