"""Where the end-to-end time of one config-3 batch goes (host pods -> picks on the host):
upload (pack + H2D), run (kernels, synchronised), picks download.  Diagnostic."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402

nodes, pods = synth.make_config(3)
pods = pods.normalized()
y = Yoda(0)
y.upload_nodes(nodes)
for _ in range(3):
    y.eval(pods, MODE_SCV)
rows = []
for _ in range(10):
    t0 = time.perf_counter()
    y.upload_pods(pods)
    t1 = time.perf_counter()
    y.run(MODE_SCV)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    y.download_picks()
    t3 = time.perf_counter()
    rows.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3))
r = np.median(np.array(rows), axis=0)
print(f"upload {r[0]:.3f} ms, run {r[1]:.3f} ms, picks download {r[2]:.3f} ms, total {r.sum():.3f}")
