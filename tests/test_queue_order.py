"""Greedy queue order (sort.go:8-10: scv/priority descending, then input index) as the host
session computes it (libyoda yoda_gs_create / yoda_gs_queue_order, pure host code): the
counting sort over small priority ranges and the stable sort over wide ones must both equal
a stable argsort of -priority, and the oracle's order (oracle_queue_order)."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import GreedySession


def _session_order(pods, nodes):
    g = GreedySession(nodes, pods, 0)
    try:
        return g.queue_order().astype(np.int64)
    finally:
        g.close()


@pytest.mark.parametrize("kind", ["small", "negative", "wide", "equal", "one"])
def test_queue_order_matches_stable_sort(kind):
    rng = np.random.default_rng(3)
    nodes = synth.make_nodes(16, seed=2)
    p = 1 if kind == "one" else 20_000
    pods = synth.make_pods(p, seed=4, priorities=True)
    if kind == "negative":  # a small span around zero (the counting sort's offset)
        pods.priority = rng.integers(-5, 6, size=p).astype(np.int64)
    elif kind == "wide":  # a span >= 2^16: the stable-sort branch
        pods.priority = rng.integers(-(1 << 40), 1 << 40, size=p).astype(np.int64)
        pods.priority[::7] = 12345  # ties across the wide range keep input order
    elif kind == "equal":
        pods.priority = np.full(p, -9, np.int64)
    want = np.argsort(-pods.priority, kind="stable")
    got = _session_order(pods, nodes)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, np.asarray(oracle.queue_order(pods), np.int64))
