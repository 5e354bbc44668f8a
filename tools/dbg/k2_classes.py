#!/usr/bin/env python3
"""Block-kernel work classes of one config-3 style batch on the GPU (device counters).
    python tools/dbg/k2_classes.py [--pods 100000] [--nodes 100000] [--config 3]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "kubernetes-scheduler_amd"))
from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--pods", type=int, default=None)
ap.add_argument("--nodes", type=int, default=None)
a = ap.parse_args()
nodes, pods = synth.make_config(a.config, pods=a.pods, nodes=a.nodes)
y = Yoda(0)
y.upload_nodes(nodes)
y.upload_pods(pods)
y.run(MODE_SCV)
y.class_stats(True)
y.run(MODE_SCV)
y.class_stats(False)
print(json.dumps(y.class_stats(), indent=1))
y.close()

if os.environ.get("YODA_K2_TRACE"):
    import numpy as np
    y = Yoda(0)
    y.upload_nodes(nodes)
    y.upload_pods(pods)
    y.run(MODE_SCV)
    y.class_stats(True)
    y.run(MODE_SCV)
    y.class_stats(False)
    tr = y.k2_trace(int(os.environ["YODA_K2_TRACE"])).astype(np.int64)
    os.makedirs("gpurun_out", exist_ok=True)
    np.save("gpurun_out/k1_trace.npy" if os.environ.get("YODA_K1_TRACE") else
            "gpurun_out/k2_trace.npy", tr)
    live = tr[:, 1] > 0
    t = tr[live]
    t0 = t[:, 0].min()
    dur = (t[:, 1] - t[:, 0]) * 10e-3  # us
    print("wave-chunks", live.sum(), "kernel span us", (t[:, 1].max() - t0) * 10e-3)
    for q in (50, 90, 99, 100):
        print(f"dur p{q} {np.percentile(dur, q):.1f} us")
    heavy = dur > np.percentile(dur, 99)
    print("heavy: npart mean", t[heavy, 2].mean(), "uni frac", t[heavy, 3].mean(),
          "start us", np.percentile((t[heavy, 0] - t0) * 10e-3, [0, 50, 100]))
    print("corr(dur, npart)", np.corrcoef(dur, t[:, 2])[0, 1])
    cls = t[:, 3]
    for name, sel in (("G", (cls & 2) != 0), ("dec uniform", ((cls & 4) != 0) & ((cls & 1) != 0)),
                      ("dec several sets", ((cls & 4) != 0) & ((cls & 1) == 0)),
                      ("unpruned", (cls & 6) == 0)):
        if sel.any():
            d = dur[sel]
            print(f"{name}: {sel.sum()} wave-chunks, dur mean {d.mean():.1f} p99 {np.percentile(d, 99):.1f} "
                  f"max {d.max():.1f} us, sum {d.sum():.0f} us, npart mean {t[sel, 2].mean():.1f}")
    ends = np.sort((t[:, 1] - t0) * 10e-3)
    print("end-time percentiles us", [round(float(np.percentile(ends, q)), 1) for q in (50, 90, 99, 99.9, 100)])
