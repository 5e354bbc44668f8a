#!/usr/bin/env python3
"""One-GPU rehearsal of the sharded greedy (BASELINE config 5 is defined on 8 GPUs; this box
has one): libyoda's own driver (yoda_comm_greedy_local = yoda_comm_greedy's protocol over the
in-process transport) with the nodes split over `world` handles on the same device, at full
size (1M pods x 100k nodes), both flags.  Reports the driver's work counters -- windows, pods
evaluated one by one (one cross-shard exchange each), capacity restarts, mid-window list
refreshes, collective calls -- and the wall time, which is NOT an 8-GPU number (the shards
share one GPU and the host-staged transport); checks every pick against the oracle digests
(tests/golden/fullsize.json) and the single-handle yoda_greedy.

    python tools/greedy_rehearsal.py --worlds 2 3 > profiles/r04/greedy_rehearsal.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-scheduler_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]

from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda, comm_greedy_local  # noqa: E402
from yoda_amd.dist import shard_bounds  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--flags", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--no-single", action="store_true",
                    help="skip the single-handle reference run (kernel-trace probes of the "
                         "sharded windows alone; the oracle digests still check every pick)")
    args = ap.parse_args()
    nodes, pods = synth.make_config(5, pods=args.pods, nodes=args.nodes)
    full = args.pods is None and args.nodes is None
    one = Yoda(0)
    one.upload_nodes(nodes)
    ref = {}
    for flags in ([] if args.no_single else args.flags):
        t0 = time.perf_counter()
        ref[flags] = one.greedy(pods, MODE_SCV, flags)
        w, f = one.greedy_stats()
        print(json.dumps({"world": 1, "flags": flags, "driver": "yoda_greedy",
                          "seconds": time.perf_counter() - t0, "windows": w, "exact_pods": f,
                          "restarts": one.greedy_restarts() if flags else 0,
                          "refreshes": one.greedy_refreshes()}), flush=True)
    one.close()
    for world in args.worlds:
        b = shard_bounds(nodes.n_nodes, world)
        hs = [Yoda(0) for _ in range(world)]
        for r, h in enumerate(hs):
            h.upload_nodes(nodes.slice(int(b[r]), int(b[r + 1])), node_offset=int(b[r]))
        for flags in args.flags:
            comm_greedy_local(hs, nodes, pods.slice(0, 4096), MODE_SCV, flags)  # warm-up
            t0 = time.perf_counter()
            pick = comm_greedy_local(hs, nodes, pods, MODE_SCV, flags)
            dt = time.perf_counter() - t0
            rec = {"world": world, "flags": flags, "driver": "yoda_comm_greedy_local",
                   "seconds": dt, **hs[0].comm_greedy_stats(),
                   "picks_equal_single_handle": (bool(np.array_equal(pick, ref[flags]))
                                                  if flags in ref else None)}
            if full:
                import fullsize_check as fc
                import oracle
                fx = fc.load_optional(f"config5_{flags}")
                if fx is not None:
                    order = oracle.queue_order(pods)
                    bad = fc.greedy_mismatch(fx, pick, nodes, pods, order, oracle)
                    rec["oracle_digests"] = "all windows match" if bad is None else bad
            print(json.dumps(rec), flush=True)
        for h in hs:
            h.close()


if __name__ == "__main__":
    main()
