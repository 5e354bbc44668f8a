import sys, time, os
sys.path[:0]=[os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'kubernetes-scheduler_amd')]
import torch
from yoda_amd import synth
from yoda_amd.capi import Yoda
nodes, pods = synth.make_config(5, pods=int(sys.argv[1]))
y = Yoda(0); y.upload_nodes(nodes)
y.greedy(pods.slice(0, 2000), 0, 1)
t0=time.perf_counter(); pk = y.greedy(pods, 0, 1); dt=time.perf_counter()-t0
print("pods", pods.n_pods, "s", dt, y.greedy_stats(times=True), "restarts", y.greedy_restarts(), flush=True)
