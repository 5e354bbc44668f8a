set -o pipefail
AB=$(realpath kubernetes-scheduler_amd/yoda_amd/libyoda_ab.so)
O=gpurun_out/r06h; mkdir -p $O
bash tools/knob_sweep.sh "-|YODA_CHUNK_ROUNDS1=8|YODA_CHUNK_ROUNDS1=10|YODA_CHUNK_ROUNDS1=12|YODA_CHUNK_ROUNDS1=16" 100000 2 > $O/sweep.txt 2>&1 || exit 1
for k in 6 8 12; do
  echo "ROUNDS1=$k" >> $O/variants.txt
  YODA_LIB_PATH=$AB YODA_CHUNK_ROUNDS1=$k timeout -k 10 300 python3 -u tools/variants.py mixed50 bytes het100k --steps 5 >> $O/variants.txt 2>> $O/variants.err || exit 1
  YODA_LIB_PATH=$AB YODA_CHUNK_ROUNDS1=$k timeout -k 10 300 python3 -u bench.py --workload greedy --steps 1 --warmup 0 --no-cpu-baseline >> $O/greedy.txt 2>> $O/greedy.err || exit 1
done
