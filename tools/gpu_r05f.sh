set -o pipefail
O=gpurun_out/r05f; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 600 bash tools/ab_run.sh 3 "r8|abl/cur.so|" "r4|abl/cur.so|YODA_CHUNK_ROUNDS2=4" "r2|abl/cur.so|YODA_CHUNK_ROUNDS2=2" "r1|abl/cur.so|YODA_CHUNK_ROUNDS2=1" "k1r4|abl/cur.so|YODA_CHUNK_ROUNDS1=4" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 400 python bench.py --workload greedy > $O/bench_greedy.json 2> $O/bench_greedy.err || { tail -20 $O/bench_greedy.err; exit 1; }
cut -c1-1200 $O/bench_greedy.json
timeout -k 10 450 bash tools/greedy_rank_probe.sh $O/rank8 0 1 || { tail -5 $O/rank8/rehearsal.err; exit 1; }
cut -c1-400 $O/rank8/rehearsal.jsonl
