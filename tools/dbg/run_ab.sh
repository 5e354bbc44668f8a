set -o pipefail
bash tools/gpu_quick.sh gpurun_out/abB "" || exit 1
bash tools/ab_lib.sh "abl/lib_A.so abl/lib_B.so" 2 || exit 1
for l in abl/lib_A.so abl/lib_B.so; do
  echo -n "$l greedy: "
  YODA_LIB_PATH=$(realpath $l) timeout -k 10 300 python bench.py --workload greedy --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('flags0', round(d['seconds'],3), d['host_times_ms'], 'cap', round(d['capacity']['seconds'],3), d['capacity']['host_times_ms'])" || exit 1
done
bash tools/dbg/gcap_env_ab.sh "YODA_WIT_CHUNK_NODES=64 YODA_WIT_CHUNK_NODES=2048 YODA_TOPK_MIN_CHUNK=1024"
