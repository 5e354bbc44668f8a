#!/usr/bin/env python3
"""Per-rank step time of pod sharding (bench.py --gpus N default), measured on ONE GPU.

For each world size W and partition kind, every rank's pod shard is timed alone against the
whole config-3 node snapshot (what each GPU of an N-GPU node runs, no collective), so the
predicted whole-job rate is P*N / max_rank(step time).  Run on a GPU box:
    python tools/pod_shard_timing.py [--steps 10] > gpurun_out/pod_shard_timing.txt
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "kubernetes-scheduler_amd"))

import torch  # noqa: E402

from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.dist import pod_partition  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--kinds", default="key256,key64,contig")
    ap.add_argument("--reverse", action="store_true", help="time the ranks last to first")
    ap.add_argument("--all-ranks", action="store_true", help="node shards: time every rank")
    args = ap.parse_args()
    nodes, pods = synth.make_config(3)
    P, N = pods.n_pods, nodes.n_nodes
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    y = Yoda(0)
    y.upload_nodes(nodes)
    y.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for W in [int(w) for w in args.worlds.split(",")]:
        for kind, by_key, block, snake in (("key256", True, 256, False),
                                           ("snake256", True, 256, True),
                                           ("key64", True, 64, False),
                                           ("contig", False, 256, False)):
            if kind not in args.kinds.split(","):
                continue
            per_rank = []
            parts = pod_partition(pods, W, by_key=by_key, block=block, snake=snake)
            ranks = list(range(W))[::-1] if args.reverse else list(range(W))
            for r in ranks:
                idx = parts[r]
                y.upload_pods(pods.take(idx))
                y.run(MODE_SCV)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    y.run(MODE_SCV)
                torch.cuda.synchronize(dev)
                per_rank.append((time.perf_counter() - t0) / args.steps * 1e3)
                if W >= 4 and len(per_rank) >= 2 and not by_key:
                    break  # contiguous parts are statistically alike; two suffice
            worst = max(per_rank)
            print(f"W={W} {kind:6s} ms/step per rank: "
                  f"{' '.join(f'{t:.3f}' for t in (per_rank[::-1] if args.reverse else per_rank))}  max {worst:.3f}  "
                  f"-> {P * N / (worst / 1e3):.3e} pairs/s", flush=True)
        if "nodes" in args.kinds.split(","):
            # node sharding's per-rank kernels (no collectives): all pods x one node block
            from yoda_amd.dist import shard_bounds
            b = shard_bounds(N, W)
            y.upload_pods(pods)
            per_rank = []
            for r in ((list(range(W))[::-1] if args.reverse else list(range(W))) if args.all_ranks else (0, W - 1)):
                y.upload_nodes(nodes.slice(int(b[r]), int(b[r + 1])), node_offset=int(b[r]))
                y.run(MODE_SCV)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    y.run(MODE_SCV)
                torch.cuda.synchronize(dev)
                per_rank.append((time.perf_counter() - t0) / args.steps * 1e3)
            if args.all_ranks and not args.reverse:
                from yoda_amd.dist import balanced_bounds
                nb = balanced_bounds(b, per_rank)
                bal = []
                for r in range(W):
                    y.upload_nodes(nodes.slice(int(nb[r]), int(nb[r + 1])),
                                   node_offset=int(nb[r]))
                    y.run(MODE_SCV)
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    for _ in range(args.steps):
                        y.run(MODE_SCV)
                    torch.cuda.synchronize(dev)
                    bal.append((time.perf_counter() - t0) / args.steps * 1e3)
                print(f"W={W} nodes  balanced bounds {list(map(int, nb))}: "
                      f"{' '.join(f'{t:.3f}' for t in bal)}  max {max(bal):.3f}", flush=True)
            print(f"W={W} nodes  ms/step ranks {'all' if args.all_ranks else '0, W-1'} "
                  f"(kernels only, no merge): "
                  f"{' '.join(f'{t:.3f}' for t in per_rank)}", flush=True)
            y.upload_nodes(nodes)
    y.close()


if __name__ == "__main__":
    main()
