set -o pipefail
O=gpurun_out/r05g; rm -rf $O; mkdir -p $O
timeout -k 10 600 bash tools/ab_run.sh 3 "cur|abl/cur.so|" "noword|abl/noword.so|" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
for spec in "cur|" "tkdec0|YODA_TOPK_DEC=0" "tkgb0|YODA_TOPK_GBEST=0" "both0|YODA_TOPK_DEC=0 YODA_TOPK_GBEST=0"; do
  IFS='|' read -r lab envs <<< "$spec"
  env YODA_LIB_PATH=$(realpath abl/cur.so) $envs timeout -k 10 300 python bench.py --workload greedy --no-cpu-baseline > $O/greedy_$lab.json 2> $O/greedy_$lab.err || { tail -5 $O/greedy_$lab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/greedy_$lab.json').read().strip().splitlines()[-1]); print('$lab', round(d['seconds'],3), round(d['capacity']['seconds'],3), d['capacity']['windows'])"
done
timeout -k 10 900 bash tools/greedy_rank_probe.sh $O/rank8 0 1 || { tail -5 $O/rank8/rehearsal_*.err; exit 1; }
cat $O/rank8/rehearsal_*.jsonl | cut -c1-300
