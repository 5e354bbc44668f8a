"""Flags-0 greedy over the first argv[1] queue pods of config 5 with the window size and list
depth from the environment (YODA_GREEDY_WINDOW, YODA_GREEDY_TOPK): run under rocprofv3 to
time the window top-k K2 per launch at capacity-window sizes (diagnostic)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler_amd"))
from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402

nodes, pods = synth.make_config(5, pods=int(sys.argv[1]))
y = Yoda(0)
y.upload_nodes(nodes)
y.greedy(pods.slice(0, 2000), 0, 0)
t0 = time.perf_counter()
y.greedy(pods, 0, 0)
print("pods", pods.n_pods, "s", round(time.perf_counter() - t0, 4), y.greedy_stats(times=True),
      flush=True)
