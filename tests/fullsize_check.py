"""Every-pick parity at BASELINE's full sizes against committed oracle digests.

tests/golden/fullsize.json holds, per block of pods, a SHA-256 digest of the C oracle's
outputs (tests/golden/make_fullsize.py, run in the build container: config 3 = 100k
independent cycles, scheduler.go:158-183 + selectHost; config 5 = 1M sequential greedy
cycles, sort.go:8-10 order with the algorithm.go:299-303 assume, both flags).  The GPU tests
hash their own outputs the same way and compare every block; on a mismatch the first differing
block is re-run through the oracle here to name the pods that differ.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
if _GOLDEN not in sys.path:
    sys.path.insert(0, _GOLDEN)

import make_fullsize as mf  # noqa: E402

FIXTURE = os.path.join(_GOLDEN, "fullsize.json")


def load(key: str) -> dict:
    with open(FIXTURE) as f:
        fx = json.load(f)
    if key not in fx:  # (generated in the build container; ~35 min per greedy flag)
        import pytest
        pytest.skip(f"{key} not in {FIXTURE} yet: run tests/golden/make_fullsize.py {key}")
    return fx[key]


def load_optional(key: str) -> dict | None:
    with open(FIXTURE) as f:
        return json.load(f).get(key)


def check_inputs(fx: dict, nodes, pods):
    got = mf.input_digest(nodes, pods)
    assert got == fx["inputs"], (
        f"the generator made different inputs here ({got}) than where the fixture was made "
        f"({fx['inputs']}): numpy drift, not a kernel mismatch")


def check_variant_inputs(fx: dict, nodes, pods):
    got = mf.input_digest(nodes, pods, mode_b=fx.get("mode", 0) == 1)
    assert got == fx["inputs"], (
        f"the generator made different inputs here ({got}) than where the fixture was made "
        f"({fx['inputs']}): numpy drift, not a kernel mismatch")


def eval_mismatch(fx: dict, got, nodes, pods, oracle, threads: int = 16) -> str | None:
    """None when every 1,024-pod block's digest matches (pick, status, feasible count, ties,
    top score and, in Mode A, the maxima of EVERY pod); else a report on the first block that
    differs, with the oracle re-run on that block."""
    mode = fx.get("mode", 0)
    dg = mf.eval_digests(got, fx["block"], mode)
    if len(dg) != len(fx["digests"]):
        return f"{len(dg)} blocks, fixture has {len(fx['digests'])}"
    bad = [b for b, (x, y) in enumerate(zip(dg, fx["digests"])) if x != y]
    if not bad:
        return None
    b = bad[0]
    B = fx["block"]
    sel = np.arange(b * B, min(pods.n_pods, (b + 1) * B))
    want = oracle.schedule(nodes, pods.take(sel), mode, threads=threads)
    ok = want.status == 0
    diffs = []
    for f in ("pick", "status", "n_feasible", "n_ties", "top_score", "maxima"):
        if f == "maxima" and mode != 0:
            continue
        g, w = getattr(got, f)[sel], getattr(want, f)
        if f in ("n_ties", "top_score"):
            g, w = np.where(ok, g, 0), np.where(ok, w, 0)
        d = np.nonzero((g != w).reshape(len(sel), -1).any(axis=1))[0]
        if d.size:
            diffs.append(f"{f}: {d.size} pods, first pod {sel[d[0]]}: gpu {g[d[0]]} oracle {w[d[0]]}")
    return (f"{len(bad)} of {len(dg)} blocks differ; first block {b}: "
            + ("; ".join(diffs) or "oracle re-run agrees with the GPU (digest drift?)"))


config3_mismatch = eval_mismatch


def greedy_mismatch(fx: dict, pick, nodes, pods, order, oracle, threads: int = 16) -> str | None:
    """None when every 6,144-pod queue window's digest matches; else the first differing pod
    of the first differing window, from the oracle re-run over that window on the state the
    earlier (matching) windows leave."""
    W = fx["window"]
    dg = mf.greedy_window_digests(pick, order, W)
    if len(dg) != len(fx["digests"]):
        return f"{len(dg)} windows, fixture has {len(fx['digests'])}"
    bad = [w for w, (x, y) in enumerate(zip(dg, fx["digests"])) if x != y]
    if not bad:
        return None
    w = bad[0]
    q0, q1 = w * W, min(pods.n_pods, (w + 1) * W)
    alloc = np.array(nodes.alloc_memory, np.uint64)
    cardn = np.array(nodes.card_number, np.uint64)
    mf.apply_assumes(alloc, cardn, pods, order[:q0], np.asarray(pick)[order[:q0]], fx["flags"])
    snap = nodes.slice(0, nodes.n_nodes)
    snap.alloc_memory = alloc
    snap.card_number = cardn
    want, *_ = oracle.greedy_mt(snap, pods, fx["flags"], q0, q1, threads=threads)
    seg = order[q0:q1]
    d = np.nonzero(np.asarray(pick)[seg] != want[seg])[0]
    where = (f"first differing queue position {q0 + d[0]} (pod {seg[d[0]]}): gpu "
             f"{pick[seg[d[0]]]} oracle {want[seg[d[0]]]}, {d.size} pods of the window"
             if d.size else "oracle re-run agrees with the GPU (digest drift?)")
    return f"{len(bad)} of {len(dg)} windows differ; first window {w}: {where}"
