"""GPU: the sharded paths that round 2 refused -- the exact NormalizeScore (K3) of U64 pods on
node shards, the greedy batch on the U64 path across shards, and libyoda's own sharded greedy
driver (yoda_comm_greedy: RCCL or the in-process transport), against the single handle and the
oracle."""
import numpy as np
import pytest

import oracle
import pyoracle as po
from yoda_amd import synth
from yoda_amd.capi import Yoda, comm_greedy_local, comm_run_local, comm_unique_id
from yoda_amd.soa import MODE_DISKIO, MODE_SCV

from test_gpu_parity import assert_same
from test_oracle import H, _overflow_pair

pytestmark = pytest.mark.gpu


def _overflow_cluster(n_other=40):
    """The two overflow nodes of tests/test_oracle.py (clock / MaxBandwidth with MaxBandwidth
    1: raw scores ~100 * clock) plus ordinary nodes, and pods that can reach them: the U64
    path, with NormalizeScore overflowing int64 for some pods (STATUS_SCORE_RANGE, or a
    wrapped in-range tie) and ordinary pods beside them."""
    scvs = []
    for clock0 in (10 ** 15 + 1, (1 << 62) // 100):
        scvs += _overflow_pair(clock0)
    rng = np.random.default_rng(5)
    for i in range(n_other):
        scvs.append(po.Scv(card_number=2, card_list=[H(int(rng.integers(1000, 30000)), clock=1500, bw=1),
                                                     H(int(rng.integers(1000, 30000)), clock=1500, bw=1)],
                           free_memory_sum=20000, total_memory_sum=64000,
                           alloc_memory=int(rng.integers(0, 30000))))
    pods = [po.Pod(), po.Pod(number=1), po.Pod(memory=5000), po.Pod(number=2, memory=1000),
            po.Pod(clock=1500), po.Pod(number=1, clock=1), po.Pod(memory=20000, number=2)]
    pods = pods * 30
    return oracle.from_py(scvs, pods, max_cards=2)


def test_overflow_cluster_needs_exact_normalize():
    nodes, pods = _overflow_cluster()
    want = oracle.schedule(nodes, pods, MODE_SCV)
    assert (want.status == po.STATUS_SCORE_RANGE).any()  # the cluster does exercise K3
    y = Yoda(0)
    y.upload_nodes(nodes)
    assert y.generic
    assert_same(y.eval(pods, MODE_SCV), want)
    y.close()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_comm_local_exact_normalize(world):
    """yoda_comm_run_local on the U64 path with overflow pods: the exact-normalize records of
    every shard all-gathered and merged (exchange 3) == the single handle == the oracle."""
    nodes, pods = _overflow_cluster()
    want = oracle.schedule(nodes, pods, MODE_SCV)
    b = np.linspace(0, nodes.n_nodes, world + 1).astype(int)
    hs = [Yoda(0) for _ in range(world)]
    for r, h in enumerate(hs):
        h.upload_nodes(nodes.slice(b[r], b[r + 1]), node_offset=int(b[r]), force_generic=True)
        h.upload_pods(pods)
    comm_run_local(hs, MODE_SCV)
    for h in hs:
        assert_same(h.download(), want)
        h.close()


@pytest.mark.parametrize("world", [2, 3])
def test_torch_exchange_exact_normalize(world):
    """The torch-driven node-shard exchange (dist.ShardExchange) with overflow pods: the same
    record exchange through Reducer.gather_tensors."""
    import torch
    from yoda_amd.dist import ShardExchange
    nodes, pods = _overflow_cluster()
    want = oracle.schedule(nodes, pods, MODE_SCV)
    b = np.linspace(0, nodes.n_nodes, world + 1).astype(int)
    hs, shards = [], []
    for r in range(world):
        y = Yoda(0)
        shards.append(nodes.slice(b[r], b[r + 1]))
        y.upload_nodes(shards[-1], node_offset=int(b[r]), force_generic=True)
        y.upload_pods(pods)
        hs.append(y)
    ex = ShardExchange.local(hs, torch.device("cuda:0"), shards, [int(x) for x in b[:-1]])
    assert_same(ex.run(MODE_SCV), want)
    for y in hs:
        y.close()


def _shard_handles(nodes, world, **kw):
    b = np.linspace(0, nodes.n_nodes, world + 1).astype(int)
    hs = []
    for r in range(world):
        y = Yoda(0)
        y.upload_nodes(nodes.slice(b[r], b[r + 1]), node_offset=int(b[r]), **kw)
        hs.append(y)
    return hs


@pytest.mark.parametrize("flags", [0, 1])
@pytest.mark.parametrize("path", ["n32", "f64", "u64"])
@pytest.mark.parametrize("world", [1, 3])
def test_comm_greedy_local(flags, path, world):
    """libyoda's sharded greedy driver (yoda_comm_greedy_local: windows, merged candidate
    lists, exact fallbacks / capacity restarts over the in-process transport) == the
    sequential oracle; the shards' node state is restored afterwards."""
    P, N = (2500, 900) if path != "u64" else (150, 300)
    nodes, pods = synth.make_config(5, pods=P, nodes=N)
    kw = {"force_f64": path == "f64", "force_generic": path == "u64"}
    hs = _shard_handles(nodes, world, **kw)
    got = comm_greedy_local(hs, nodes, pods, MODE_SCV, flags)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, flags)
    np.testing.assert_array_equal(got, want)
    # restored: the same batch again gives the same picks
    np.testing.assert_array_equal(comm_greedy_local(hs, nodes, pods, MODE_SCV, flags), want)
    for y in hs:
        y.close()


def test_comm_greedy_rccl_world1():
    """yoda_comm_greedy over a one-rank RCCL communicator == yoda_greedy, both flags, and
    Mode B."""
    nodes, pods = synth.make_config(5, pods=3000, nodes=1200)
    y = Yoda(0)
    y.upload_nodes(nodes)
    y.comm_init(comm_unique_id(), 0, 1)
    for flags in (0, 1):
        np.testing.assert_array_equal(y.comm_greedy(nodes, pods, MODE_SCV, flags),
                                      y.greedy(pods, MODE_SCV, flags))
    np.testing.assert_array_equal(y.comm_greedy(nodes, pods, MODE_DISKIO, 0),
                                  y.greedy(pods, MODE_DISKIO, 0))
    y.close()


@pytest.mark.parametrize("flags", [0, 1])
def test_sharded_greedy_u64(flags):
    """dist.sharded_greedy on the U64 record path (every pod one exact sharded step) ==
    the sequential oracle."""
    import torch
    from yoda_amd.dist import HandleShard, Reducer, sharded_greedy
    nodes, pods = synth.make_config(5, pods=120, nodes=300)
    hs = _shard_handles(nodes, 2, force_generic=True)
    dev = torch.device("cuda:0")
    got = sharded_greedy([HandleShard(h, dev) for h in hs], Reducer(local=True), nodes, pods,
                         flags)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, flags)
    np.testing.assert_array_equal(got, want)
    for y in hs:
        y.close()


@pytest.mark.parametrize("flags", [0, 1])
def test_comm_greedy_local_windows_vs_oracle(flags):
    """The config-5 generator at 14,000 pods x 8,000 nodes (several 6,144-pod windows, the
    mid-window list refresh in flags 0, capacity restarts in flags 1) over three node shards
    with libyoda's driver: every pick equals the sequential oracle's."""
    nodes, pods = synth.make_config(5, pods=14_000, nodes=8_000)
    hs = _shard_handles(nodes, 3)
    got = comm_greedy_local(hs, nodes, pods, MODE_SCV, flags)
    st = hs[0].comm_greedy_stats()
    assert st["windows"] >= 3
    np.testing.assert_array_equal(got, oracle.greedy_mt(nodes, pods, flags, threads=16)[0])
    for y in hs:
        y.close()
