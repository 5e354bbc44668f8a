#!/usr/bin/env python3
"""Step time of the hot path on the workloads the headline does not cover (GPU box).

Each variant: upload, warm up, time `--steps` yoda_run steps (HIP-event K1/K2 split), one run
with the class counters on, and optionally the first `--check` pods against the C oracle
(picks, statuses, ties, feasible counts).  One JSON object per variant on stdout.

    python tools/variants.py [names...] [--steps 5] [--check 256]
names: yoda_amd/synth.py VARIANTS (default: all but mixed100 and c4diskio)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "kubernetes-scheduler_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.soa import MODE_DISKIO, MODE_SCV  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--check", type=int, default=0)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    names = args.names or ["c3", "mixed50", "bytes", "u64", "c4", "het100k", "diskio",
                          "diskio_distinct"]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    for name, nodes, pods, mode, kw in synth.variant_workloads(names):
        y = Yoda(0)
        y.upload_nodes(nodes, **kw)
        y.upload_pods(pods)
        y.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        y.run(mode)
        torch.cuda.synchronize(dev)
        y.profile(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            y.run(mode)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        y.profile(False)
        k1, k2, nl = y.profile_read()
        out = {"variant": name, "pods": pods.n_pods, "nodes": nodes.n_nodes, "path": y.path,
               "mode": "diskio" if mode == MODE_DISKIO else "scv", "ms_per_step": ms,
               "pairs_per_s": pods.n_pods * nodes.n_nodes / (ms / 1e3),
               "k1_ms": k1 / max(nl, 1), "k2_ms": k2 / max(nl, 1)}
        if mode == MODE_SCV and y.path == "n32":
            y.class_stats(True)
            y.run(mode)
            torch.cuda.synchronize(dev)
            y.class_stats(False)
            out["classes"] = y.class_stats()
        res = y.download()
        out["status_counts"] = {str(s): int((res.status == s).sum()) for s in np.unique(res.status)}
        if args.check:
            import oracle
            n = min(args.check, pods.n_pods)
            idx = np.linspace(0, pods.n_pods - 1, n).astype(np.int64)
            sub = pods.take(idx)
            t0 = time.perf_counter()
            want = oracle.schedule(nodes, sub, mode, threads=args.threads)
            ok = all(np.array_equal(getattr(res, f)[idx], getattr(want, f))
                     for f in ("pick", "status", "n_ties", "n_feasible"))
            out["check"] = {"pods": n, "match": bool(ok), "oracle_s": time.perf_counter() - t0}
        y.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
