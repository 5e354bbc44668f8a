set -o pipefail
O=gpurun_out/r05d; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
YODA_SEED_DEBUG=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/bench_dbg.json 2> $O/bench_dbg.err || { tail $O/bench_dbg.err; exit 1; }
grep seeds $O/bench_dbg.err | tail -1
python3 -c "import json; d=json.loads(open('$O/bench_dbg.json').read().strip().splitlines()[-1]); print(d['extra']['classes']['k2_blocks'], {k: round(v['ms_per_step'],3) for k,v in d['extra']['variants'].items()})"
timeout -k 10 900 bash tools/ab_run.sh 3 "cur|abl/cur.so|" "nodeseed|abl/nodeseed.so|" "nodec|abl/cur.so|YODA_KB_DEC=0" "nogbest|abl/cur.so|YODA_GBEST=0" "noseed|abl/cur.so|YODA_SEEDS=0" "nolv|abl/cur.so|YODA_KB_LEVELS=0" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
