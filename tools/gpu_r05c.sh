set -o pipefail
O=gpurun_out/r05c; rm -rf $O; mkdir -p $O
YODA_SEED_DEBUG=1 timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --steps 2 --warmup 1 > $O/seed_debug.json 2> $O/seed_debug.err || { tail $O/seed_debug.err; exit 1; }
grep seeds $O/seed_debug.err | tail -2
timeout -k 10 900 bash tools/ab_run.sh 3 "ab7|abl/ab7.so|" "ab7ns|abl/ab7ns.so|" "ab5|abl/ab5.so|" "ab5ns|abl/ab5ns.so|" "ab7_noseed|abl/ab7.so|YODA_SEEDS=0" "ab7_nolv|abl/ab7.so|YODA_KB_LEVELS=0" "ab5ns_noseed|abl/ab5ns.so|YODA_SEEDS=0 YODA_KB_LEVELS=0" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
