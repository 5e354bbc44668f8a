set -o pipefail
bash tools/ab.sh YODA_CHUNK_ROUNDS1 "2 3 4 6" 2 > gpurun_out/ab_r1.txt 2>&1 || exit 1
cat gpurun_out/ab_r1.txt
bash tools/ab.sh YODA_CHUNK_ROUNDS2 "4 8 12 16" 2 > gpurun_out/ab_r2.txt 2>&1 || exit 1
cat gpurun_out/ab_r2.txt
