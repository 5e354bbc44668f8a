"""GPU: node-shard evaluation with the exchange in the caller's pod order (yoda_shard_exchange_
order, and yoda_comm_run on the fast paths): every shard sorts its pods with the padded
counting order and its nodes in the block-grouped order of yoda_run (shards of >= 4096 one-model
nodes), the exchanged maxima / counts / keys / ties are scattered to the caller's order and
gathered back.  Against the oracle, and against the shared radix order."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda, comm_run_local
from yoda_amd.soa import MODE_DISKIO, MODE_SCV

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def workload():
    nodes, pods = synth.make_config(3, pods=6000, nodes=13000)
    want = {m: oracle.schedule(nodes, pods, m, threads=8) for m in (MODE_SCV, MODE_DISKIO)}
    return nodes, pods, want


def _handles(nodes, pods, world):
    b = np.linspace(0, nodes.n_nodes, world + 1).astype(int)
    hs, shards = [], []
    for r in range(world):
        y = Yoda(0)
        shards.append(nodes.slice(b[r], b[r + 1]))
        y.upload_nodes(shards[-1], node_offset=int(b[r]))
        y.upload_pods(pods)
        hs.append(y)
    return hs, shards, [int(x) for x in b[:-1]]


@pytest.mark.parametrize("world", [1, 2, 3])
def test_comm_local_caller_order(workload, world):
    nodes, pods, want = workload
    hs, _, _ = _handles(nodes, pods, world)
    assert all(h.node_order_grouped for h in hs)   # >= 4096 one-model nodes per shard
    for mode in (MODE_SCV, MODE_DISKIO, MODE_SCV):
        comm_run_local(hs, mode)
        for h in hs:
            assert_same(h.download(), want[mode], mode)
    info = hs[0].order_info()
    assert info["kind"] == 2 and info["work"] >= pods.n_pods   # the padded counting order
    for h in hs:
        h.close()


@pytest.mark.parametrize("caller_order", [True, False])
def test_torch_exchange_orders(workload, caller_order):
    import torch
    from yoda_amd.dist import ShardExchange
    nodes, pods, want = workload
    hs, shards, offs = _handles(nodes, pods, 2)
    ex = ShardExchange.local(hs, torch.device("cuda:0"), shards, offs, caller_order=caller_order)
    for mode in (MODE_DISKIO, MODE_SCV):
        assert_same(ex.run(mode), want[mode], mode)
    # the last (Mode A) run: counting order with caller-order exchange, else the radix order
    assert hs[0].order_info()["kind"] == (2 if caller_order else 1)
    for y in hs:
        y.close()


def test_greedy_window_refuses_caller_order():
    """The greedy windows' top-k reads the shared radix order: a caller-order phase 1 is
    refused there with a named error rather than mixing orders."""
    from yoda_amd.capi import YodaError
    nodes, pods = synth.make_config(5, pods=600, nodes=5000)
    y = Yoda(0)
    y.upload_nodes(nodes)
    y.upload_pods(pods)
    y.shard_exchange_order(True)
    import torch
    from yoda_amd.dist import ShardBuffers
    b = ShardBuffers(pods.n_pods, torch.device("cuda:0"))
    y.shard_phase1(MODE_SCV, ShardBuffers.ptr(b.maxima), ShardBuffers.ptr(b.counts))
    with pytest.raises(YodaError, match="caller-order"):
        y.shard_topk(ShardBuffers.ptr(b.maxima), ShardBuffers.ptr(b.counts))
    y.close()
