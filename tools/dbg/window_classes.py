"""Block-kernel classes and K1/K2 times of one greedy-sized window of config 5 (the first W
pods in queue order) evaluated as an ordinary batch, for W in argv (diagnostic)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402

nodes, pods = synth.make_config(5, pods=200_000)
order = np.argsort(-pods.priority, kind="stable")
y = Yoda(0)
y.upload_nodes(nodes)
for W in [int(a) for a in sys.argv[1:]] or [512, 4096, 16384]:
    idx = order[:W]
    sub = pods.slice(0, W)
    for f in ("has_number", "number", "has_memory", "memory", "has_clock", "clock", "priority",
              "rio", "rcpu"):
        setattr(sub, f, getattr(pods, f)[idx])
    y.eval(sub, MODE_SCV)
    y.profile(True)
    for _ in range(5):
        y.eval(sub, MODE_SCV)
    torch.cuda.synchronize()
    k1, k2, n = y.profile_read()
    y.profile(False)
    y.class_stats(True)
    y.eval(sub, MODE_SCV)
    y.class_stats(False)
    print(json.dumps({"W": W, "k1_us": 1e3 * k1 / max(n, 1), "k2_us": 1e3 * k2 / max(n, 1),
                      "classes": y.class_stats()}))
