set -o pipefail
mkdir -p gpurun_out
for w in 4096 8192 16384 2048; do
YODA_GREEDY_WINDOW=$w timeout -k 10 300 python bench.py --workload greedy > gpurun_out/gw_$w.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/gw_$w.json').read().strip().splitlines()[-1]); print('window $w', round(d['seconds'],4), 's', d['windows'], 'windows', d['exact_fallback_pods'], 'fallbacks', {k: round(v,1) for k,v in d['host_times_ms'].items()}, 'match', d['cpu_baseline']['sample_picks_match_gpu'])"
done
