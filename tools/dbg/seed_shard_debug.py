#!/usr/bin/env python3
"""Debug: the foreign-maxima shard cluster of tests/test_gpu_shard_seeds.py -- per shard the
K2 work classes and the mismatches against the oracle (run once per libyoda build)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("kubernetes-scheduler_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from test_gpu_shard_seeds import split_maxima_cluster  # noqa: E402
from yoda_amd.capi import Yoda, comm_run_local  # noqa: E402

nodes, pods, split = split_maxima_cluster()
want = oracle.schedule(nodes, pods, 0, threads=8)
b = [0, split, nodes.n_nodes]
hs = [Yoda(0) for _ in range(2)]
for r, h in enumerate(hs):
    h.upload_nodes(nodes.slice(b[r], b[r + 1]), node_offset=b[r])
    h.upload_pods(pods)
for it in range(3):
    for h in hs:
        h.class_stats(True)
    comm_run_local(hs, 0)
    for h in hs:
        h.class_stats(False)
    got = hs[0].download()
    bad = np.nonzero(got.pick != want.pick)[0]
    print(f"run {it}: {len(bad)} pick mismatches; first {bad[:8].tolist()}", flush=True)
    for r, h in enumerate(hs):
        cs = h.class_stats()
        print(f"  shard {r}: k2 {cs.get('k2')} k2_blocks {cs.get('k2_blocks')} k1_blocks "
              f"{cs.get('k1_blocks')}", flush=True)
