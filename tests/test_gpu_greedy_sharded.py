"""Sharded greedy batch on one GPU: G node shards = G libyoda handles (yoda_shard_topk,
yoda_shard_best_one, yoda_set_node_state) driven by yoda_amd/dist.py sharded_greedy with the
exchange done in-process; picks == the sequential oracle (oracle_greedy)."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_SCV

pytestmark = pytest.mark.gpu


def _shards(nodes, G, path):
    import torch
    from yoda_amd.dist import HandleShard, Reducer, agree_on_path, shard_bounds
    dev = torch.device("cuda:0")
    b = shard_bounds(nodes.n_nodes, G)
    handles, parts, offs = [], [], []
    for g in range(G):
        y = Yoda(0)
        parts.append(nodes.slice(int(b[g]), int(b[g + 1])))
        offs.append(int(b[g]))
        y.upload_nodes(parts[-1], node_offset=offs[-1], force_f64=path == "f64")
        handles.append(y)
    red = Reducer(local=True)
    agree_on_path(red, handles, parts, offs, dev)
    return handles, [HandleShard(h, dev) for h in handles], red


@pytest.mark.parametrize("G", [1, 3])
@pytest.mark.parametrize("path", ["n32", "f64"])
def test_sharded_greedy_matches_oracle(G, path):
    from yoda_amd.dist import sharded_greedy
    nodes, pods = synth.make_config(5, pods=9000, nodes=700)
    handles, shards, red = _shards(nodes, G, path)
    stats = {}
    got = sharded_greedy(shards, red, nodes, pods, 0, 4096, stats)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, 0)
    np.testing.assert_array_equal(got, want)
    assert stats["windows"] == 3 and stats["exact_pods"] > 0
    if G == 1:  # the snapshot is restored: a fresh batch still matches the oracle
        sub = pods.slice(0, 200)
        np.testing.assert_array_equal(handles[0].eval(sub, MODE_SCV).pick,
                                      oracle.schedule(nodes, sub, MODE_SCV, threads=8).pick)
    for h in handles:
        h.close()


def test_sharded_greedy_card_capacity():
    from yoda_amd.dist import sharded_greedy
    nodes, pods = synth.make_config(5, pods=300, nodes=400)
    handles, shards, red = _shards(nodes, 2, "n32")
    got = sharded_greedy(shards, red, nodes, pods, 1)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, 1)
    np.testing.assert_array_equal(got, want)
    for h in handles:
        h.close()


def test_sharded_greedy_drivers_same_windows():
    """Capacity windows: dist.sharded_greedy (torch-side driver) and yoda_comm_greedy_local
    (libyoda's own) take the same deep lists through the same merge (yoda_shard_topk_deep,
    yoda_merge_shard_lists), so they run the same window sequence -- equal window and restart
    counts -- and both equal the oracle."""
    from yoda_amd.capi import comm_greedy_local
    from yoda_amd.dist import sharded_greedy
    nodes, pods = synth.make_config(5, pods=4000, nodes=3000)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, 1)
    handles, shards, red = _shards(nodes, 3, "n32")
    stats = {}
    got = sharded_greedy(shards, red, nodes, pods, 1, stats=stats)
    np.testing.assert_array_equal(got, want)
    lib_pick = comm_greedy_local(handles, nodes, pods, MODE_SCV, 1)
    np.testing.assert_array_equal(lib_pick, want)
    st = handles[0].comm_greedy_stats()
    assert (stats["windows"], stats["restarts"]) == (st["windows"], st["restarts"]), (stats, st)
    for h in handles:
        h.close()


def test_sharded_greedy_equals_single_handle():
    from yoda_amd.dist import sharded_greedy
    nodes, pods = synth.make_config(5, pods=6000, nodes=900)
    one = Yoda(0)
    one.upload_nodes(nodes)
    single = one.greedy(pods, MODE_SCV, 0)
    one.close()
    handles, shards, red = _shards(nodes, 4, "n32")
    np.testing.assert_array_equal(sharded_greedy(shards, red, nodes, pods, 0), single)
    for h in handles:
        h.close()


def test_set_node_state_matches_oracle():
    """yoda_set_node_state (sparse assume) == a snapshot with that allocated memory."""
    nodes, pods = synth.make_config(2, pods=300, nodes=1500)
    y = Yoda(0)
    y.upload_nodes(nodes)
    rng = np.random.default_rng(3)
    sel = rng.choice(nodes.n_nodes, 200, replace=False).astype(np.uint32)
    alloc = nodes.alloc_memory.copy()
    alloc[sel] += rng.integers(0, 60000, sel.size).astype(np.uint64)
    y.set_node_state(sel, alloc[sel], nodes.card_number[sel])
    mod = nodes.slice(0, nodes.n_nodes)
    mod.alloc_memory = alloc
    want = oracle.schedule(mod, pods, MODE_SCV, threads=8)
    got = y.eval(pods, MODE_SCV)
    np.testing.assert_array_equal(got.pick, want.pick)
    np.testing.assert_array_equal(got.top_score[want.status == 0],
                                  want.top_score[want.status == 0])
    y.close()
