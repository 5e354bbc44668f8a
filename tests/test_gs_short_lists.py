"""Greedy session with lists that end before the pod's feasible count (round 5).

The capacity windows' lists are merged deeper than the chunks' lists and end where they are no
longer certain to be exact (k_topk_merge_deep): entries past that point are empty (node
0xffffffff).  The session (libyoda yoda_gs_*, pure host code) must then take the last listed
entry as the threshold and must not treat the list as the whole feasible set, even when the
feasible count fits the list depth.  Reference: the sequential assume of config 5
(scheduler.go Score over the current node state; DESIGN.md §5 "Greedy, round 5").
"""
import numpy as np

from yoda_amd import synth
from yoda_amd.capi import GreedySession

EMPTY = 0xFFFFFFFF


def _pods(n, memory):
    pods = synth.make_pods(n, seed=5)
    pods.has_memory[:] = 1
    pods.memory[:] = memory
    pods.has_clock[:] = 0
    pods.has_number[:] = 0
    pods.priority[:] = 0
    return pods


def _window(g, k, nf, lists):
    """Window of len(lists) pods from queue position 0; lists: [(score, node), ...] per pod."""
    wn = len(lists)
    counts = np.zeros(2 * wn, np.uint32)
    counts[:wn] = nf
    ts = np.full((k, wn), -1.0)
    ti = np.full((k, wn), EMPTY, np.uint32)
    for i, lst in enumerate(lists):
        for kk, (s, n) in enumerate(lst):
            ts[kk, i], ti[kk, i] = s, n
    g.begin_window(0, k, counts, ts.ravel(), ti.ravel())


def test_short_list_is_not_whole():
    nodes = synth.make_nodes(8, seed=2)
    # a large request: the first pick's Allocate score drops, so its node falls below the
    # second pod's threshold (its only listed entry)
    pods = _pods(2, int(nodes.total_memory_sum.max()) // 2)
    g = GreedySession(nodes, pods, 0)
    try:
        # both pods: 3 feasible nodes, a 4-deep list holding only node 0 (score 1000)
        _window(g, 4, 3, [[(1000.0, 0)], [(1000.0, 0)]])
        nxt = g.resolve()
        # pod 0 is certified (node 0 untouched: its score is the threshold, lowest index);
        # pod 1's node 0 now scores below it and nodes 1, 2 are unlisted: not certified
        assert nxt == 1
        pick, _, _ = g.picks()
        assert pick[0] == 0
    finally:
        g.close()


def test_whole_list_still_certifies():
    nodes = synth.make_nodes(8, seed=2)
    pods = _pods(2, int(nodes.total_memory_sum.max()) // 2)
    g = GreedySession(nodes, pods, 0)
    try:
        # the same window with every feasible node listed: the list is the feasible set, so the
        # second pod picks its best current candidate without a threshold
        _window(g, 4, 3, [[(1000.0, 0), (900.0, 1), (800.0, 2)]] * 2)
        assert g.resolve() == 2
    finally:
        g.close()
