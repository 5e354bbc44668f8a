"""Config 5 at its full size (BASELINE.json: 1M pods x 100k nodes greedy), both greedy modes.

  0. EVERY pick against the sequential C oracle (sort.go:8-10 order, algorithm.go:299-303
     assume, plus the CardNumber decrement with YODA_GREEDY_CARD_CAPACITY): the oracle's 1M
     cycles run in the build container (tests/golden/make_fullsize.py, ~35 min per flag on 8
     cores); tests/golden/fullsize.json holds one digest per 6,144-pod queue window, which the
     GPU's picks must reproduce window by window;
  1. exact picks against oracle_greedy run here on a queue-order prefix of 2,000 pods -- a
     prefix in queue order is an exact sub-problem;
  2. replay at sampled queue positions across the whole batch: the node state just before
     position q is rebuilt from the earlier picks (allocated memory += scv/memory, CardNumber
     -= the pod's number), uploaded to a second handle, and that pod alone is scheduled on it
     (an independent scheduling cycle, yoda_eval): the pick must be the greedy's;
  3. every pick is feasible against the running state (PodFitsNumber on the decremented
     CardNumber; memory/clock predicates do not change), and each node's final allocated
     memory equals its start value plus the scv/memory of the pods assigned to it.
"""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_SCV

pytestmark = pytest.mark.gpu

CAP = 1  # YODA_GREEDY_CARD_CAPACITY


@pytest.fixture(scope="module")
def cfg5():
    nodes, pods = synth.make_config(5)
    order = oracle.queue_order(pods)
    return nodes, pods, order


def _replay_state(nodes, pods, order, pick, q, flags):
    """(alloc, card_number) just before queue position q."""
    done = order[:q]
    pk = pick[done]
    ok = pk >= 0
    idx = pk[ok].astype(np.int64)
    alloc = np.array(nodes.alloc_memory, np.uint64)
    mem = np.where(pods.has_memory[done][ok] == 1, pods.memory[done][ok], 0).astype(np.uint64)
    np.add.at(alloc, idx, mem)  # uint64 wrap, like Go
    cn = np.array(nodes.card_number, np.uint64)
    if flags & CAP:
        num = np.where(pods.has_number[done][ok] == 1, pods.number[done][ok], 1).astype(np.uint64)
        dec = np.zeros(nodes.n_nodes, np.uint64)
        np.add.at(dec, idx, num)
        assert (dec <= cn).all()  # a pick needs number <= CardNumber: no saturation
        cn = cn - dec
    return alloc, cn


@pytest.mark.parametrize("flags", [0, CAP])
def test_config5_full_size(cfg5, flags):
    nodes, pods, order = cfg5
    P = pods.n_pods
    y = Yoda(0)
    y.upload_nodes(nodes)
    pick = y.greedy(pods, MODE_SCV, flags)
    windows, restarts = y.greedy_stats()
    assert windows >= P // 6144  # windows of at most kGreedyWindow pods (yoda_capi.cpp)
    if flags == 0:
        # the mid-window list refresh ran (the replays below sample the windows it served)
        assert y.greedy_refreshes() > 0

    # 0. every pick, window by window, against the oracle's digests
    import fullsize_check as fc
    fx = fc.load_optional(f"config5_{flags}")
    assert fx is not None, f"config5_{flags} digests missing: tests/golden/make_fullsize.py"
    fc.check_inputs(fx, nodes, pods)
    bad = fc.greedy_mismatch(fx, pick, nodes, pods, order, oracle)
    assert bad is None, bad
    assert int((pick >= 0).sum()) == fx["placed"]

    # 1. exact prefix against the sequential oracle
    pre = order[:2000]
    want, _ = oracle.greedy(nodes, pods.take(pre), MODE_SCV, flags)
    np.testing.assert_array_equal(pick[pre], want)

    # 3. feasibility against the running state, and the allocated-memory balance
    num_eff = np.where(pods.has_number == 1, pods.number, 1).astype(np.uint64)
    cn = np.array(nodes.card_number, np.uint64)
    pk_q = pick[order]
    assert (pk_q >= -2).all() and (pk_q < nodes.n_nodes).all()
    placed = pk_q >= 0
    if flags & CAP:
        for p, n in zip(order[placed], pk_q[placed]):
            assert num_eff[p] <= cn[n] or (pods.has_number[p] and pods.number[p] == 0)
            cn[n] -= num_eff[p]
    else:
        assert (num_eff[order[placed]] <= cn[pk_q[placed]]).all()
    alloc_end, cn_end = _replay_state(nodes, pods, order, pick, P, flags)
    if flags & CAP:
        np.testing.assert_array_equal(cn_end, cn)
    mem = np.where(pods.has_memory == 1, pods.memory, 0).astype(np.uint64)
    per_node = np.zeros(nodes.n_nodes, np.uint64)
    np.add.at(per_node, pick[pick >= 0].astype(np.int64), mem[pick >= 0])
    np.testing.assert_array_equal(alloc_end - np.array(nodes.alloc_memory, np.uint64), per_node)

    # 2. replay: one independent cycle at sampled queue positions across the batch
    rng = np.random.default_rng(17 + flags)
    # window boundaries (6144-pod windows) and their neighbours, where a window's candidate
    # lists give way to the next window's
    wb = np.array([6144 * k + d for k in (1, 40, 120) for d in (-1, 0, 1)])
    # and the first two windows, where the flags-0 fallbacks and list refreshes cluster
    qs = np.unique(np.concatenate([[0, 2000, P // 2, P - 1], wb[wb < P],
                                   rng.integers(0, P, size=8), rng.integers(0, 2 * 6144, size=12)]))
    two = Yoda(0)
    for q in qs:
        alloc, cnq = _replay_state(nodes, pods, order, pick, int(q), flags)
        snap = nodes.slice(0, nodes.n_nodes)
        snap.alloc_memory = alloc
        snap.card_number = cnq
        two.upload_nodes(snap)
        p = int(order[q])
        res = two.eval(pods.take([p]), MODE_SCV)
        assert int(res.pick[0]) == int(pick[p]), (q, p)
    two.close()
    # the uploaded snapshot is unchanged afterwards
    sub = pods.slice(0, 64)
    np.testing.assert_array_equal(y.eval(sub, MODE_SCV).pick,
                                  oracle.schedule(nodes, sub, MODE_SCV, threads=8).pick)
    y.close()


@pytest.mark.parametrize("flags", [0, CAP])
def test_config5_generator_several_windows_vs_oracle(flags):
    """The config-5 generator at 14,000 pods x 8,000 nodes: more than two 6144-pod windows
    (window boundaries, exact fallbacks / capacity restarts across them), every pick against
    the sequential oracle."""
    nodes, pods = synth.make_config(5, pods=14_000, nodes=8_000)
    y = Yoda(0)
    y.upload_nodes(nodes)
    pick = y.greedy(pods, MODE_SCV, flags)
    windows, _ = y.greedy_stats()
    assert windows >= 3
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, flags)
    np.testing.assert_array_equal(pick, want)
    y.close()
