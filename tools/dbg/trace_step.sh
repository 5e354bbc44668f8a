#!/bin/bash
# rocprofv3 kernel trace of a short bench run; prints one step's kernel sequence.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/tstep
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --no-extras --steps 4 --warmup 1 > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
python3 - $OUT <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
k1=[i for i,r in enumerate(rows) if 'k1_block' in r['Kernel_Name']]
a,b=k1[2],k1[3]
tot=0
for r in rows[a:b]:
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    tot+=d
    print(r['Kernel_Name'][:60].ljust(60), '%.1f'%d)
print('sum %.1f us; wall %.1f us' % (tot, (int(rows[b]['Start_Timestamp'])-int(rows[a]['Start_Timestamp']))/1e3))
PY
