#!/usr/bin/env python3
"""Per-rank step time of bench.py --gpus W, measured on ONE GPU, for both shardings.

What rank r of a W-GPU run executes, timed alone (the collectives' latency is not in it; the
model in DESIGN.md §7 adds it):
  pods   (bench.py --shard pods): the whole config-3 node snapshot and pod part r of
         dist.pod_partition; a private yoda_run, nothing exchanged;
  nodes  (bench.py --shard nodes, the north_star's RCCL merge): all 100k pods and node block r
         of dist.shard_bounds through the torch-driven shard step (dist.ShardExchange: shard
         phase 1, the maxima/count merge, shard phase 2, the packed-key merge, finalize), with
         the one-rank local reducer standing in for the all-reduces;
  nodes_lib  the same through libyoda's own exchange (yoda_comm_run_local with one handle:
         device copies in place of the RCCL collectives, bench.py --exchange libyoda).
One JSON line per (kind, W): per-rank ms/step (wall, HIP-synchronised), per-rank K1 / K2
HIP-event ms, and the predicted whole-job pairs/s at max over ranks.

    python tools/rank_probe.py [--worlds 1,2,4,8] [--kinds pods,nodes] [--steps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "kubernetes-scheduler_amd"))

import torch  # noqa: E402

from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.dist import ShardExchange, pod_partition, shard_bounds  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402


def timed(y, step, dev, steps):
    step()
    torch.cuda.synchronize(dev)
    y.profile(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    y.profile(False)
    k1, k2, nl = y.profile_read()
    return ms, k1 / max(nl, 1), k2 / max(nl, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--kinds", default="pods,nodes,nodes_lib")
    args = ap.parse_args()
    nodes, pods = synth.make_config(3)
    P, N = pods.n_pods, nodes.n_nodes
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    kinds = args.kinds.split(",")
    for W in [int(w) for w in args.worlds.split(",")]:
        if "pods" in kinds:
            y = Yoda(0)
            y.upload_nodes(nodes)
            y.set_stream(stream)
            rows = []
            for part in pod_partition(pods, W):
                y.upload_pods(pods.take(part))
                rows.append(timed(y, lambda: y.run(MODE_SCV), dev, args.steps))
            y.close()
            emit("pods", W, P, N, rows)
        if "nodes_lib" in kinds:  # the same shard step through libyoda's own exchange
            from yoda_amd.capi import comm_run_local
            b = shard_bounds(N, W)
            rows = []
            for r in range(W):
                lo, hi = int(b[r]), int(b[r + 1])
                y = Yoda(0)
                y.upload_nodes(nodes.slice(lo, hi), node_offset=lo)
                y.upload_pods(pods)
                y.set_stream(stream)
                rows.append(timed(y, lambda: comm_run_local([y], MODE_SCV), dev, args.steps))
                y.close()
            emit("nodes_lib", W, P, N, rows)
        if "nodes" in kinds:
            b = shard_bounds(N, W)
            rows = []
            for r in range(W):
                lo, hi = int(b[r]), int(b[r + 1])
                y = Yoda(0)
                shard = nodes.slice(lo, hi)
                y.upload_nodes(shard, node_offset=lo)
                y.upload_pods(pods)
                ex = ShardExchange.local([y], dev, [shard], [lo])
                rows.append(timed(y, lambda: ex.step(MODE_SCV), dev, args.steps))
                y.close()
            emit("nodes", W, P, N, rows)


def emit(kind, W, P, N, rows):
    worst = max(r[0] for r in rows)
    print(json.dumps({"kind": kind, "world": W, "ms_per_rank": [r[0] for r in rows],
                      "k1_ms": [r[1] for r in rows], "k2_ms": [r[2] for r in rows],
                      "max_ms": worst, "pairs_per_s_at_max": P * N / (worst / 1e3)}),
          flush=True)


if __name__ == "__main__":
    main()
