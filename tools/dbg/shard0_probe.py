"""Is node shard 0's extra time (8 ranks) tied to its data or to node_offset 0?"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "kubernetes-scheduler_amd"))
import numpy as np, torch
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_SCV

nodes, pods = synth.make_config(3)
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
y = Yoda(0); y.set_stream(torch.cuda.current_stream(dev).cuda_stream)
y.upload_pods(pods)
def t(sl, off, label):
    y.upload_nodes(sl, node_offset=off); y.run(MODE_SCV); torch.cuda.synchronize(dev)
    y.profile(True)
    t0 = time.perf_counter()
    for _ in range(10): y.run(MODE_SCV)
    torch.cuda.synchronize(dev)
    y.profile(False); k1, k2, n = y.profile_read()
    print(f"{label:40s} {(time.perf_counter()-t0)/10*1e3:.3f} ms  k1 {k1/n:.3f} k2 {k2/n:.3f}", flush=True)
s0, s7 = nodes.slice(0, 12500), nodes.slice(87500, 100000)
t(s0, 0, "shard0 data, offset 0")
t(s0, 87500, "shard0 data, offset 87500")
t(s7, 0, "shard7 data, offset 0")
t(s7, 87500, "shard7 data, offset 87500")
t(nodes.slice(1, 12501), 1, "nodes [1,12501)")
t(nodes.slice(6250, 18750), 6250, "nodes [6250,18750)")
y.close()
