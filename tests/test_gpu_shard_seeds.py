"""GPU: node shards whose local card maxima (the G table) are below the run's global PreScore
maxima.  The K2 pruning seeds are scores under this handle's G; they are
lower bounds of a pod's scores only when the pod's maxima are this handle's own.  After an
exchange the maxima can exceed a shard's G (another shard holds the fastest GPU model), the pod's
real scores on this shard drop below the seed, and a seeded K2 would prune its true best.

The cluster: shard 0 holds a few nodes of the fastest model (bandwidth 2000, ...) with almost no
free memory and no allocatable memory, so they set the maxima of every pod that fits them (pods
with no scv/memory and no conflicting scv/clock) but never win; the rest of shard 0 has
CardNumber 0 (infeasible).  Shard 1 holds models 0/1 only and every winner.  Reference:
collection.go:30-55 (maxima over every SCV), algorithm.go:264-291 (scores under them)."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda, comm_run_local
from yoda_amd.soa import MODE_SCV

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def split_maxima_cluster(n=4000, fast=160, p=1500, seed=3):
    """(nodes, pods, split): shard 0 = [0, split) holds the fast-model nodes, shard 1 the rest."""
    nodes = synth.make_nodes(n, seed=seed, cards=8)
    pods = synth.make_pods(p, seed=seed + 1)
    split = n // 2
    k = nodes.card_clock.shape[1]
    f = slice(0, fast)
    nodes.card_clock[f] = synth.CLOCKS[2]
    nodes.card_bandwidth[f] = synth.BANDWIDTHS[2]
    nodes.card_core[f] = synth.CORES[2]
    nodes.card_power[f] = synth.POWERS[2]
    nodes.card_total_memory[f] = synth.TOTALS[2]
    nodes.card_free_memory[f] = np.random.default_rng(seed).integers(0, 48, (fast, k))
    nodes.card_healthy[f] = 1
    nodes.free_memory_sum[f] = nodes.card_free_memory[f].sum(axis=1)
    nodes.total_memory_sum[f] = nodes.card_total_memory[f].sum(axis=1)
    nodes.alloc_memory[f] = nodes.total_memory_sum[f]      # Allocate 0
    dead = slice(fast, split)                               # CardNumber 0: never feasible
    nodes.card_number[dead] = 0
    # shard 1: every node model 1 (one-model 64-node blocks, which the block K1 needs to seed
    # K2's threshold; their free memory rescaled to model 1's total)
    rest = slice(split, n)
    real = nodes.card_total_memory[rest] > 0
    for arr, table in ((nodes.card_clock, synth.CLOCKS), (nodes.card_bandwidth, synth.BANDWIDTHS),
                       (nodes.card_core, synth.CORES), (nodes.card_power, synth.POWERS),
                       (nodes.card_total_memory, synth.TOTALS)):
        arr[rest] = np.where(real, table[1], 0).astype(np.uint64)
    fr = nodes.card_free_memory[rest]
    fr = np.minimum(fr, synth.TOTALS[1]).astype(np.uint64)
    t = nodes.card_total_memory[rest]
    nodes.card_free_memory[rest] = fr
    nodes.free_memory_sum[rest] = fr.sum(axis=1)
    nodes.total_memory_sum[rest] = t.sum(axis=1)
    nodes.alloc_memory[rest] = np.minimum(nodes.alloc_memory[rest], nodes.total_memory_sum[rest])
    return nodes.normalized(), pods, split


def test_cluster_exercises_foreign_maxima():
    """The precondition, on the oracle: many pods take their bandwidth maximum from shard 0's
    fast nodes and still pick a node of shard 1."""
    nodes, pods, split = split_maxima_cluster()
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    foreign = (want.status == 0) & (want.maxima[:, 0] == synth.BANDWIDTHS[2]) & \
        (want.pick >= split)
    assert foreign.sum() >= 100, int(foreign.sum())


@pytest.mark.parametrize("world", [2, 3])
def test_comm_local_foreign_maxima(world):
    """libyoda's sharded step (yoda_comm_run_local) on shards whose G is below the global
    maxima == the oracle, pod by pod."""
    nodes, pods, split = split_maxima_cluster()
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    b = [0, split, nodes.n_nodes] if world == 2 else [0, split, split + 1000, nodes.n_nodes]
    hs = [Yoda(0) for _ in range(world)]
    for r, h in enumerate(hs):
        h.upload_nodes(nodes.slice(b[r], b[r + 1]), node_offset=int(b[r]))
        h.upload_pods(pods)
    assert all(h.path == "n32" for h in hs)
    for _ in range(2):  # (twice: a second run on the same handles)
        comm_run_local(hs, MODE_SCV)
        for h in hs:
            assert_same(h.download(), want)
    for h in hs:
        h.close()


def test_torch_exchange_foreign_maxima():
    """The torch-driven exchange (dist.ShardExchange: yoda_shard_phase1 / phase2) on the same
    shards == the oracle."""
    import torch
    from yoda_amd.dist import ShardExchange
    nodes, pods, split = split_maxima_cluster()
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    b = [0, split, nodes.n_nodes]
    hs, shards = [], []
    for r in range(2):
        y = Yoda(0)
        shards.append(nodes.slice(b[r], b[r + 1]))
        y.upload_nodes(shards[-1], node_offset=b[r])
        y.upload_pods(pods)
        hs.append(y)
    ex = ShardExchange.local(hs, torch.device("cuda:0"), shards, b[:-1])
    assert_same(ex.run(MODE_SCV), want)
    for y in hs:
        y.close()
