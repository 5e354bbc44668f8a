#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz).

The reference cannot run here (pure Go, no toolchain), so the expected outputs come from
the C oracle (oracle/yoda_oracle.c), cross-checked at generation time against the
independent Python restatement (oracle/pyoracle.py).  They pin the oracle and libyoda
against regressions; they are NOT reference-produced vectors.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "kubernetes-scheduler_amd"), os.path.join(REPO, "oracle"),
                os.path.dirname(HERE)]

import oracle  # noqa: E402
import pyoracle as po  # noqa: E402
from yoda_amd import synth  # noqa: E402

NODE_FIELDS = ["card_number", "card_count", "free_memory_sum", "total_memory_sum",
               "alloc_memory", "card_free_memory", "card_total_memory", "card_clock",
               "card_bandwidth", "card_core", "card_power", "card_healthy", "cpu", "disk_io"]
POD_FIELDS = ["has_number", "number", "has_memory", "memory", "has_clock", "clock", "priority",
              "rio", "rcpu"]
OUT_FIELDS = ["pick", "status", "n_feasible", "n_ties", "top_score", "maxima"]


def edge_cluster():
    rng = np.random.default_rng(2024)
    nodes = synth.make_nodes(120, seed=2025, cards=4)
    nodes.card_number[::7] = 0
    nodes.card_clock[rng.random(nodes.card_clock.shape) < 0.3] = 1500
    nodes.total_memory_sum[5] = 0
    nodes.alloc_memory[::11] = np.uint64((1 << 64) - 7)       # > Total: Allocate = 0
    pods = synth.make_pods(40, seed=2026)
    pods.has_number[:4] = 1
    pods.number[:4] = [0, (1 << 64) - 1, 3, 16]                  # "0", "-1", 3, 16
    pods.has_memory[4:8] = 1
    pods.memory[4:8] = [0, (1 << 64) - 5, 81920, 1]
    pods.has_clock[8:12] = 1
    pods.clock[8:12] = [1500, 1 << 40, 0, 1410]
    pods.rio[12:16] = [0.0, np.inf, -np.inf, np.float32(0.1)]
    pods.rcpu[12:16] = [0, 100, 500, -100]
    return nodes.normalized(), pods.normalized()


def cases():
    from test_oracle import kat1_cluster, _overflow_pair
    scvs, pod = kat1_cluster()
    yield "kat1", oracle.from_py(scvs, [pod])
    yield "config1", synth.make_config(1)
    yield "config2_small", synth.make_config(2, pods=64, nodes=400)
    yield "config4_small", synth.make_config(4, pods=64, nodes=400)
    yield "edges", edge_cluster()
    yield "overflow", oracle.from_py(_overflow_pair(10 ** 15 + 1) + _overflow_pair((1 << 62) // 100),
                                     [po.Pod(), po.Pod(number=1)])


def main():
    for name, (nodes, pods) in cases():
        nodes, pods = nodes.normalized(), pods.normalized()
        arrays = {f"node_{f}": getattr(nodes, f) for f in NODE_FIELDS}
        arrays.update({f"pod_{f}": getattr(pods, f) for f in POD_FIELDS})
        scvs, plist = oracle.to_py(nodes, pods)
        for mode in (0, 1):
            res = oracle.schedule(nodes, pods, mode)
            for p, pod in enumerate(plist):          # cross-check with the Python restatement
                r = po.schedule_one(pod, scvs, mode)
                assert (int(res.pick[p]), int(res.status[p])) == (r.pick, r.status), (name, p)
            for f in OUT_FIELDS:
                arrays[f"mode{mode}_{f}"] = getattr(res, f)
        for flags in (0, 1):
            pick, status = oracle.greedy(nodes, pods, 0, flags)
            assert list(map(int, pick)) == po.greedy(plist, scvs, 0, card_capacity=bool(flags))
            arrays[f"greedy{flags}_pick"] = pick
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        print(name, nodes.n_nodes, "nodes", pods.n_pods, "pods")


if __name__ == "__main__":
    main()
