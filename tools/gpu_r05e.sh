set -o pipefail
O=gpurun_out/r05e; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
YODA_K2_TRACE=60000 timeout -k 10 200 python tools/dbg/k2_classes.py > $O/k2_trace.txt 2>&1 || { tail $O/k2_trace.txt; exit 1; }
tail -16 $O/k2_trace.txt
timeout -k 10 600 bash tools/ab_run.sh 3 "cur|abl/cur.so|" "noz|abl/cur.so|YODA_NODE_ZORDER=0" "nodec|abl/cur.so|YODA_KB_DEC=0" "nogbest|abl/cur.so|YODA_GBEST=0" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
