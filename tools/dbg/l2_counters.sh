set -o pipefail
mkdir -p gpurun_out/l2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/l2/a -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1 > $R/gpurun_out/l2/a.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $R/gpurun_out/l2/b -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1 > $R/gpurun_out/l2/b.log 2>&1
cd $R
python3 - <<'PY'
import csv, glob, collections
for d in ("a", "b"):
    f = glob.glob(f"gpurun_out/l2/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no file", d); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0][-30:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, m in agg.items():
        if "k2_block" in k or "k1_block" in k:
            print(d, k, {c: f"{sum(v)/len(v):.4g}" for c, v in m.items()})
PY
