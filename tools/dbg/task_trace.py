#!/usr/bin/env python3
"""Per-(wave, chunk) task durations of the block K1 or K2 on one batch (GPU box).

The kernels stamp each task's start / end with s_memrealtime (100 MHz) when YODA_K2_TRACE=<slots>
is set (YODA_K1_TRACE=1: the K1 records instead of the K2).  Prints the task count, the duration
distribution, the kernel's span, the mean concurrency (sum of task durations / span) and the
durations split by per-pod work (npart = 0: the task's fixed cost plus its lane = block pass).

    YODA_K2_TRACE=200000 [YODA_K1_TRACE=1] python tools/dbg/task_trace.py [--pods P] [--nodes N]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "kubernetes-scheduler_amd"))
import numpy as np  # noqa: E402

from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=None)
ap.add_argument("--nodes", type=int, default=None)
ap.add_argument("--variant", default=None, help="a synth.VARIANTS name instead of config 3")
a = ap.parse_args()
slots = int(os.environ.get("YODA_K2_TRACE", "0"))
if slots <= 0:
    raise SystemExit("set YODA_K2_TRACE=<slots> (and YODA_K1_TRACE=1 for K1)")
kern = "k1" if os.environ.get("YODA_K1_TRACE") else "k2"
if a.variant:
    _, nodes, pods, _, kw = next(synth.variant_workloads([a.variant]))
else:
    nodes, pods = synth.make_config(3, pods=a.pods, nodes=a.nodes)
    kw = {}
y = Yoda(0)
y.upload_nodes(nodes, **kw)
y.upload_pods(pods)
y.run(MODE_SCV)
y.run(MODE_SCV)
y.class_stats(True)
y.run(MODE_SCV)
y.class_stats(False)
tr = y.k2_trace(slots)
y.close()
used = tr[:, 1] > 0
# slots another launch of the batch wrote and the last one did not (a different grid shape):
# keep the tasks of the last launch only (those that started within 5 ms of the last start)
if used.any():
    t0_last = tr[used][:, 0].astype(np.int64).max()
    used &= tr[:, 0].astype(np.int64) >= t0_last - 500000
t = tr[used].astype(np.int64)
dur = (t[:, 1] - t[:, 0]) / 100.0  # us at 100 MHz
span = (t[:, 1].max() - t[:, 0].min()) / 100.0
npart = t[:, 2] & 0xffffffff
nblk = t[:, 2] >> 32  # K1: blocks classified node by node
q = lambda v, x: float(np.percentile(v, x)) if len(v) else None  # noqa: E731
out = {"kernel": kern, "tasks": int(used.sum()), "span_us": span,
       "mean_concurrency": float(dur.sum() / span) if span > 0 else None,
       "dur_us": {"mean": float(dur.mean()), "p10": q(dur, 10), "p50": q(dur, 50),
                  "p90": q(dur, 90), "p99": q(dur, 99), "max": float(dur.max())},
       "npart0": {"tasks": int((npart == 0).sum()), "mean_us": float(dur[npart == 0].mean())
                  if (npart == 0).any() else None},
       "npart_pos": {"tasks": int((npart > 0).sum()), "mean_us": float(dur[npart > 0].mean())
                     if (npart > 0).any() else None, "mean_npart": float(npart[npart > 0].mean())
                     if (npart > 0).any() else None},
       "corr_dur_npart": float(np.corrcoef(dur, npart)[0, 1]) if len(dur) > 2 else None}
if kern == "k1" and len(dur) > 3:
    # least squares: task duration ~ a + b * node-by-node blocks + c * PART nodes
    A = np.stack([np.ones(len(dur)), nblk, npart], axis=1).astype(np.float64)
    coef = np.linalg.lstsq(A, dur, rcond=None)[0]
    out["fit_us"] = {"base": float(coef[0]), "per_node_block": float(coef[1]),
                     "per_part_node": float(coef[2])}
    out["node_blocks"] = {"mean": float(nblk.mean()), "sum": int(nblk.sum())}
    out["span_share"] = {"base": float(coef[0] * len(dur) / dur.sum()),
                         "node_blocks": float(coef[1] * nblk.sum() / dur.sum()),
                         "part": float(coef[2] * npart.sum() / dur.sum())}
# phases (the trace's word 3): K1 set-up end | block-pass end << 32; K2 flags | set-up end << 16 |
# block-list walk end << 40 (ticks after the task's start)
w3 = tr[used][:, 3].astype(np.uint64)
if kern == "k1":
    t_set = (w3 & np.uint64(0xffffffff)).astype(np.int64) / 100.0
    t_pass = (w3 >> np.uint64(32)).astype(np.int64) / 100.0
else:
    t_set = ((w3 >> np.uint64(16)) & np.uint64(0xffffff)).astype(np.int64) / 100.0
    t_pass = ((w3 >> np.uint64(40)) & np.uint64(0xffffff)).astype(np.int64) / 100.0
out["phase_us_mean"] = {"setup": float(t_set.mean()), "pass": float((t_pass - t_set).mean()),
                        "epilogue": float((dur - t_pass).mean())}
z = npart == 0
if z.any():
    out["phase_us_mean_npart0"] = {"setup": float(t_set[z].mean()),
                                   "pass": float((t_pass[z] - t_set[z]).mean()),
                                   "epilogue": float((dur[z] - t_pass[z]).mean())}
if kern == "k2":  # task time by wave kind: G waves, decoupled-bound (non-G) waves, others
    fl = w3 & np.uint64(0xffff)
    for name, sel in (("g", (fl & np.uint64(2)) != 0), ("dec", (fl & np.uint64(4)) != 0),
                      ("other", (fl & np.uint64(6)) == 0)):
        out["by_kind_" + name] = {"tasks": int(sel.sum()), "dur_sum_us": float(dur[sel].sum()),
                                  "mean_us": float(dur[sel].mean()) if sel.any() else None,
                                  "npart_sum": int(npart[sel].sum())}
# start-time profile: how many tasks start in each tenth of the span
st = (t[:, 0] - t[:, 0].min()) / 100.0
out["starts_by_tenth"] = np.histogram(st, bins=10, range=(0, span))[0].tolist()
out["ends_by_tenth"] = np.histogram((t[:, 1] - t[:, 0].min()) / 100.0, bins=10, range=(0, span))[0].tolist()
print(json.dumps(out), flush=True)
# raw records for offline analysis (TASK_TRACE_DUMP=<path.npz>): slot (= wave * chunks + chunk),
# start, end, npart, word 3
dump = os.environ.get("TASK_TRACE_DUMP")
if dump:
    np.savez_compressed(dump, slot=np.nonzero(used)[0], rec=tr[used])
