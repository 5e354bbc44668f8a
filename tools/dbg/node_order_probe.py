"""Probe: config-3 step time when the node snapshot is stored grouped (by GPU model, then by
card capacity) instead of in its input order -- the same cluster, permuted.  Timing only
(tie picks follow the storage order here).  python tools/dbg/node_order_probe.py"""
import json
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


def permuted(order):
    out = nodes.slice(0, nodes.n_nodes)
    for f in ("card_number", "card_count", "free_memory_sum", "total_memory_sum", "alloc_memory",
              "cpu", "disk_io", "card_free_memory", "card_total_memory", "card_clock",
              "card_bandwidth", "card_core", "card_power", "card_healthy"):
        setattr(out, f, np.ascontiguousarray(getattr(nodes, f)[order]))
    return out


hfs = np.sort(np.where(nodes.card_healthy == 1, nodes.card_free_memory, 0), axis=1)[:, ::-1]
clock = nodes.card_clock[:, 0]
variants = {
    "input": np.arange(nodes.n_nodes),
    "by_model": np.argsort(clock, kind="stable"),
    "by_model_hfs4": np.lexsort((hfs[:, 3], clock)),
    "by_model_hfs0": np.lexsort((hfs[:, 0], clock)),
}
y = Yoda(0)
for name, order in variants.items():
    y.upload_nodes(permuted(order))
    y.upload_pods(pods)
    for _ in range(3):
        y.run(MODE_SCV)
    torch.cuda.synchronize()
    y.profile(True)
    t0 = time.perf_counter()
    for _ in range(10):
        y.run(MODE_SCV)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10 * 1e3
    y.profile(False)
    k1, k2, n = y.profile_read()
    y.class_stats(True)
    y.run(MODE_SCV)
    y.class_stats(False)
    c = y.class_stats()
    print(json.dumps({"order": name, "ms_per_step": round(dt, 3), "k1_ms": round(k1 / n, 3),
                      "k2_ms": round(k2 / n, 3), "k1": c["k1"], "k2": c["k2"]}))
